#!/bin/bash
# One parameterised entry point for GPU-box sessions (run through gpurun):
#
#   gpurun -- 'bash scripts/gpu.sh TAG step [step ...]'
#
# Every step runs under its own time limit; the first failing step ends the
# call (no GPU work after a fault, abort or timeout).  Outputs land in
# gpurun_out/TAG/.  Steps:
#   micro[:BIN]       scripts/mb/BIN (mixed-add variants; default: all)
#   tests[:K]         pytest -m gpu (optionally -k K, commas -> spaces)
#   smoke             __graft_entry__.smoke()
#   bench[:ARGS]      python bench.py ARGS (commas -> spaces)
#   prof[:ARGS]       rocprofv3 --kernel-trace --stats around bench.py ARGS
#   pmc:CTRS[:ARGS]   one rocprofv3 --pmc pass (CTRS comma-separated) around bench.py ARGS
#   py:SCRIPT[,ARGS]  python3 scripts/SCRIPT ARGS
#   profpy:SCRIPT[,ARGS] rocprofv3 --kernel-trace --stats around python3 scripts/SCRIPT ARGS
#   bin:PATH[,ARGS]   a built binary (e.g. kzg-commitments_amd/tools/kzg_bench)
#   profbin:PATH[,ARGS] rocprofv3 --kernel-trace --stats around a built binary
#   env:VAR=VALUE     export VAR for the steps that follow (A/B switches)
#   tracebin:PATH[,ARGS] kernel + HIP runtime API trace around a built binary
#   pmcpy:CTRS:SCRIPT[,ARGS] one rocprofv3 --pmc pass around python3 scripts/SCRIPT ARGS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for st in "$@"; do
  n=$((n + 1))
  kind=${st%%:*}
  arg=""
  [[ "$st" == *:* ]] && arg=${st#*:}
  case $kind in
    micro)
      bins=${arg:-$(ls scripts/mb)}
      for b in $bins; do
        echo "== $b" >> "$OUT/micro.txt"
        timeout -k 10 120 "./scripts/mb/$b" >> "$OUT/micro.txt" 2>&1 || { echo "micro $b failed"; exit 1; }
      done
      ;;
    tests)
      k=()
      [[ -n "$arg" ]] && k=(-k "${arg//,/ }")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$OUT/tests_$n.log" 2>&1 || { tail -30 "$OUT/tests_$n.log"; exit 1; }
      tail -3 "$OUT/tests_$n.log"
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log"
      ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg//,/ } > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" \
        || { tail -20 "$OUT/bench_$n.err"; exit 1; }
      tail -c 600 "$OUT/bench_$n.json"
      ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o prof --output-format csv \
        -- python3 -u bench.py ${arg//,/ } > "$OUT/prof_$n.json" 2> "$OUT/prof_$n.err" \
        || { tail -20 "$OUT/prof_$n.err"; exit 1; }
      ;;
    pmc)
      ctrs=${arg%%:*}
      bargs=""
      [[ "$arg" == *:* ]] && bargs=${arg#*:}
      timeout -s KILL 300 rocprofv3 --pmc ${ctrs//,/ } -d "$OUT/pmc_$n" -o pmc --output-format csv \
        -- python3 -u bench.py ${bargs//,/ } > "$OUT/pmc_$n.json" 2> "$OUT/pmc_$n.err" \
        || { tail -20 "$OUT/pmc_$n.err"; exit 1; }
      ;;
    py)
      # py:SCRIPT[,ARGS] -- a script under scripts/ (commas -> spaces)
      set -- ${arg//,/ }
      timeout -k 10 600 python3 -u "scripts/$1" "${@:2}" > "$OUT/py_$n.txt" 2>&1 \
        || { tail -20 "$OUT/py_$n.txt"; exit 1; }
      tail -20 "$OUT/py_$n.txt"
      ;;
    profpy)
      # profpy:SCRIPT[,ARGS] -- rocprofv3 kernel trace + stats around a script under scripts/
      set -- ${arg//,/ }
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/profpy_$n" -o prof --output-format csv \
        -- python3 -u "scripts/$1" "${@:2}" > "$OUT/profpy_$n.txt" 2>&1 \
        || { tail -20 "$OUT/profpy_$n.txt"; exit 1; }
      tail -12 "$OUT/profpy_$n.txt"
      ;;
    bin)
      set -- ${arg//,/ }
      timeout -k 10 600 "./$1" "${@:2}" > "$OUT/bin_$n.txt" 2>&1 || { tail -20 "$OUT/bin_$n.txt"; exit 1; }
      tail -20 "$OUT/bin_$n.txt"
      ;;
    profbin)
      set -- ${arg//,/ }
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/profbin_$n" -o prof --output-format csv \
        -- "./$1" "${@:2}" > "$OUT/profbin_$n.txt" 2>&1 || { tail -20 "$OUT/profbin_$n.txt"; exit 1; }
      tail -12 "$OUT/profbin_$n.txt"
      ;;
    pmcpy)
      ctrs=${arg%%:*}
      sargs=${arg#*:}
      set -- ${sargs//,/ }
      timeout -s KILL 300 rocprofv3 --pmc ${ctrs//,/ } -d "$OUT/pmcpy_$n" -o pmc --output-format csv \
        -- python3 -u "scripts/$1" "${@:2}" > "$OUT/pmcpy_$n.txt" 2>&1 \
        || { tail -20 "$OUT/pmcpy_$n.txt"; exit 1; }
      ;;
    tracebin)
      set -- ${arg//,/ }
      timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d "$OUT/tracebin_$n" -o trace \
        --output-format csv -- "./$1" "${@:2}" > "$OUT/tracebin_$n.txt" 2>&1 || { tail -20 "$OUT/tracebin_$n.txt"; exit 1; }
      tail -12 "$OUT/tracebin_$n.txt"
      ;;
    env)
      export "${arg?}"
      echo "env $arg"
      ;;
    *)
      echo "unknown step $st"
      exit 2
      ;;
  esac
done
echo "all steps ok"
