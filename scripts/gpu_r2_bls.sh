set -o pipefail
D=gpurun_out/r2/bls
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python3 scripts/lat_micro.py > $D/lat_micro.txt 2>&1 || { tail -20 $D/lat_micro.txt; exit 1; }
grep -v amdgpu.ids $D/lat_micro.txt
timeout -k 10 600 python3 bench.py --workload cfg4 --steps 10 --warmup 2 --no-cpu-baseline --no-latency > $D/cfg4.json 2> $D/cfg4.err || { tail -20 $D/cfg4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$D/cfg4.json').read().strip().splitlines()[-1]); s=d['secondary']
print('cfg4', round(d['value']), d['config']['msm'], {k: v for k, v in s.items() if 'pip' in k or 'valu' in k or 'mixed' in k})"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -2 $D/tests.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $D/tests.log | head -30; exit $rc; }
