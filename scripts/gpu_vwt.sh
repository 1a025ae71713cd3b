# wave-verify phase timing + correctness; needs: (cd kzg-commitments_amd && make variant NAME=vwt VFLAGS=-DKZGX_VW_TIMING)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pairing.py -x -q --timeout 300 --timeout-method thread -k "verify" > gpurun_out/vwt_tests.log 2>&1; rc=$?
tail -2 gpurun_out/vwt_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/vwt_tests.log | head -20; exit 1; }
for c in BN254 BLS12381; do
KZGX_LIB=variants/vwt/libkzgx.so timeout -k 10 300 python scripts/bench_verify.py --curve $c --verifies 64 --pairings 64 > gpurun_out/vwt_$c.log 2>&1 || { tail -5 gpurun_out/vwt_$c.log; exit 1; }
grep vw_ts gpurun_out/vwt_$c.log | sort | uniq -c | sort -rn | head -2
timeout -k 10 300 python scripts/bench_verify.py --curve $c > gpurun_out/vwb_$c.json 2>&1 || { tail -5 gpurun_out/vwb_$c.json; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/vwb_$c.json').read().strip().splitlines()[-1])
print(d['curve'], 'verify_ms', {k:round(v,2) for k,v in d['verify_ms'].items()}, d['checked'])
for m,r in d['single_verify_sweep'].items(): print('  ', m, {k:(round(v['ms'],2), round(v['per_s']), v['all_ok']) for k,v in r.items()})
"
done
