"""Per-kernel register / spill table from hipcc's kernel-resource-usage remarks.

    python tools/regusage.py [TU ...]     (default: the sweep and family TUs)

Compiles each translation unit of mcmc-for-nested-data_amd/csrc device-only with the
Makefile's flags and prints one line per kernel: VGPRs, SGPRs, VGPR/SGPR spills, scratch.
"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "mcmc-for-nested-data_amd" / "csrc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fPIC",
         "-I../../include", "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"]


def usage(tu):
    # (as the Makefile: the sweep TUs and fam_linreg / fam_gauss_mean without machine LICM)
    extra = (["-mllvm", "-disable-machine-licm"]
             if tu.startswith("sweep_") or tu in ("fam_linreg", "fam_gauss_mean") else [])
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", tu + ".hip", "-o",
                        "/tmp/_regusage.o"], cwd=CSRC, capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|SGPRs|VGPRs Spill|SGPRs Spill|"
                      r"ScratchSize \[bytes/lane\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    return rows


def main():
    tus = sys.argv[1:] or ["sweep_linreg", "sweep_gauss_mean", "sweep_logistic", "fam_linreg"]
    for tu in tus:
        for r in usage(tu):
            dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
            print(f"{tu:18s} v{r.get('VGPRs','?'):>4s} s{r.get('SGPRs','?'):>4s} "
                  f"vspill {r.get('VGPRs Spill','?'):>3s} sspill {r.get('SGPRs Spill','?'):>3s} "
                  f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4s}  {dem}")


if __name__ == "__main__":
    main()
