#!/bin/bash
# GPU tests (-k filter), the bench line, phase stamps and the per-tile timeline.
TAG=${1:-g}
K=${2:-partial or scale or configs}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "$K" > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-pmc > gpurun_out/b_$TAG.json 2>gpurun_out/b_$TAG.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/b_$TAG.json'));print('value %.4g  us/iter %.3f  kernel us/launch %.0f' % (d['value'], d['ms_per_step']*1e3, d['roofline']['avg_launch_us']))"
timeout -k 10 120 python tools/stamps.py partial > gpurun_out/s_$TAG.json 2>&1 || exit $?
timeout -k 10 120 python tools/tilegantt.py > gpurun_out/g_$TAG.json 2>&1 || exit $?
python3 - <<PY
import json
s = json.load(open('gpurun_out/s_$TAG.json'))['stamps']
for k in ('blk0_w0', 'blk0_w1'):
    print(k, s[k]['iter_cycles'], s[k]['phase_cycles'], s[k].get('hyper_wait_done'), s[k].get('aux_poll_load_join_done'))
d = json.load(open('gpurun_out/g_$TAG.json'))
for st in d['tiles'][:3]:
    print('step', st['step'], 'span', st['span'], {w: [(a, b) for _, a, b in v] for w, v in st['waves'].items()})
PY
