import os, sys, numpy
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tests", "golden")); sys.path.insert(0, os.path.join(ROOT, "mcmc-for-nested-data_amd")); sys.path.insert(0, ROOT)
from gpu_cases import synthetic, partial_state, run_engine
for (C, G, N, n_iter) in [(4, 5, 40, 45), (64, 8, 64, 45), (4, 5, 40, 5)]:
    fam, sizes, _, _, _ = synthetic("linreg_partial", C, G, N)
    st, _ = partial_state(fam, sizes, C, 2)
    res = {}
    for name, env in (("kvar", {}), ("fill", {"NMC_KVAR": "0"})):
        res[name] = run_engine(fam, sizes, st, numpy.arange(C), 0, n_iter, 5, env=env, burn=0)
    a, b = res["kvar"], res["fill"]
    print(C, G, N, n_iter, a[3]["zin"], b[3]["zin"], a[3]["mode"], a[3]["waves_per_group"])
    for k, nm in ((0, "acc"), (1, "llp"), (2, "rows")):
        x, y = a[k], b[k]
        same = numpy.array_equal(x, y, equal_nan=True)
        print(" ", nm, "same" if same else "DIFF", "nan kvar", int(numpy.isnan(x).sum()) if x.dtype != numpy.uint8 else 0,
              "nan fill", int(numpy.isnan(y).sum()) if y.dtype != numpy.uint8 else 0)
        if not same and k == 2:
            bad = numpy.argwhere(~((x == y) | (numpy.isnan(x) & numpy.isnan(y))))
            print("   first diffs (chain,row,col):", bad[:6].tolist())
            r0 = bad[0][1]
            print("   kvar row", x[bad[0][0], r0, :8]); print("   fill row", y[bad[0][0], r0, :8])
        if not same and k == 1:
            bad = numpy.argwhere(~((x == y) | (numpy.isnan(x) & numpy.isnan(y))))
            print("   first llp diffs (chain,iter,p,g):", bad[:6].tolist())
