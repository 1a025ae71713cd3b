# round-2 refresh on the current tree: serial rocprof kernel stats of the
# default table path and of Pippenger (isolated kernel durations), then the
# cfg3 / cfg4 / cfg5 bench lines
set -o pipefail
O=gpurun_out/r2/s3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_serial -o run --output-format csv -- python3 bench.py --serial --steps 10 --warmup 2 --no-cpu-baseline --no-pippenger --no-latency > $O/prof_serial.json 2> $O/prof_serial.err || { echo "prof serial failed"; tail -20 $O/prof_serial.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_pip -o run --output-format csv -- python3 bench.py --fixed-bits 0 --serial --steps 5 --warmup 2 --no-cpu-baseline --no-latency > $O/prof_pip.json 2> $O/prof_pip.err || { echo "prof pip failed"; tail -20 $O/prof_pip.err; exit 1; }
for d in prof_serial prof_pip; do f=$(find $O/$d -name "*kernel_stats.csv" | head -1); cp "$f" $O/$d.kernel_stats.csv; echo "== $d"; cut -d, -f1-5 "$f" | head -10; done
timeout -k 10 400 python3 bench.py --workload cfg3 --no-pippenger --no-latency --no-cpu-baseline > $O/cfg3.json 2> $O/cfg3.err || { echo "cfg3 failed"; tail -5 $O/cfg3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg3.json')); print('cfg3', round(d['value']), round(d['ms_per_step'],3), d['config']['msm'], d['parity']['ok'])"
timeout -k 10 400 python3 bench.py --workload cfg4 --no-latency --no-cpu-baseline > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed"; tail -5 $O/cfg4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4', round(d['value']), round(d['ms_per_step'],3), d['config']['msm'], d['parity']['ok'], 'pip', round(d['secondary']['pippenger']['value']))"
timeout -k 10 400 python3 bench.py --workload cfg5 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || { echo "cfg5 failed"; tail -5 $O/cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cfg5.json')); print('cfg5', d['value'], d['ms_per_step'], d.get('parity'))"
