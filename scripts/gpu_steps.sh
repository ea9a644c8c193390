#!/bin/bash
# One parameterised GPU session (replaces the per-round gpu_r0*.sh one-offs).  Each step runs under its own
# time limit; the session stops at the first failure.  Output: gpurun_out/<tag>/.
#
#   bash scripts/gpu_steps.sh <tag> <step> [<step> ...]
#
# steps:
#   host                         host model (nproc, lscpu)
#   tests[:<pytest -k expr>]     python -m pytest tests -m gpu [-k expr]
#   smoke                        __graft_entry__.smoke()
#   bench[:<bench.py args>]      python bench.py <args>                    -> bench_<i>.json / .log
#   ab:<VAR>:<rounds>:<args>     bench.py <args> with VAR=0 and VAR=1, interleaved <rounds> times -> ab_<VAR>.txt
#   trace[:<bench.py args>]      rocprofv3 --kernel-trace --stats over bench.py <args> -> trace/, kernel_stats_by_grid.csv
#   pmc:<c1,c2,..>:<args>        one rocprofv3 --pmc pass over bench.py <args> -> pmc_<i>/ + summary
#   tool:<binary> [args]         ./tools/<binary> [args]                    -> tool_<binary>.txt
#   sh:<script> [args]           bash scripts/<script> [args]               -> sh_<i>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
T=gpurun_out/$TAG
mkdir -p "$T"
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  echo "== step $i: $step"
  case $kind in
    host)
      (nproc; lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS") > "$T/host.txt"
      ;;
    tests)
      k=()
      [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread "${k[@]}" \
        > "$T/pytest_$i.log" 2>&1 || { tail -40 "$T/pytest_$i.log"; exit 1; }
      tail -2 "$T/pytest_$i.log"
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > "$T/smoke.log" 2>&1 \
        || { tail -20 "$T/smoke.log"; exit 1; }
      tail -1 "$T/smoke.log"
      ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 600 python -u bench.py $arg > "$T/bench_$i.json" 2> "$T/bench_$i.log" || { tail -20 "$T/bench_$i.log"; exit 1; }
      grep -h "^\[" "$T/bench_$i.log" | cut -c1-400
      cut -c1-400 "$T/bench_$i.json"
      ;;
    ab)
      var=${arg%%:*}
      rest=${arg#*:}
      rounds=${rest%%:*}
      args=${rest#*:}
      for r in $(seq "$rounds"); do
        for v in 0 1; do
          echo "-- round $r $var=$v" >> "$T/ab_$var.txt"
          # shellcheck disable=SC2086
          env "$var=$v" timeout -k 10 600 python -u bench.py $args 2>&1 >/dev/null | grep "^\[" | cut -c1-700 >> "$T/ab_$var.txt" \
            || { tail -20 "$T/ab_$var.txt"; exit 1; }
        done
      done
      cat "$T/ab_$var.txt"
      ;;
    trace)
      # shellcheck disable=SC2086
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$T/trace" -o run -- \
        python3 bench.py $arg > "$T/bench_traced.json" 2> "$T/bench_traced.log" || { tail -5 "$T/bench_traced.log"; exit 1; }
      python3 scripts/stats_by_grid.py "$T/trace/run_kernel_trace.csv" > "$T/kernel_stats_by_grid.csv" || exit 1
      head -30 "$T/kernel_stats_by_grid.csv"
      ;;
    pmc)
      ctrs=${arg%%:*}
      args=${arg#*:}
      # shellcheck disable=SC2086
      timeout -s KILL 180 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d "$T/pmc_$i" -o run -- python3 bench.py $args \
        > "$T/pmc_$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$T/pmc_$i.log"; exit 1; }
      python3 scripts/summarize_pmc.py "$T/pmc_$i" > "$T/pmc_$i.txt" 2>&1
      head -40 "$T/pmc_$i.txt"
      ;;
    sh)
      # shellcheck disable=SC2086
      timeout -k 10 900 bash scripts/$arg > "$T/sh_$i.txt" 2>&1 || { tail -20 "$T/sh_$i.txt"; exit 1; }
      cat "$T/sh_$i.txt"
      ;;
    tool)
      bin=${arg%% *}
      targs=""
      [[ "$arg" == *" "* ]] && targs=${arg#* }
      # shellcheck disable=SC2086
      timeout -k 10 300 "./tools/$bin" $targs > "$T/tool_$bin.txt" 2>&1 || { tail -20 "$T/tool_$bin.txt"; exit 1; }
      cat "$T/tool_$bin.txt"
      ;;
    *)
      echo "unknown step $step"; exit 2
      ;;
  esac
done
echo "session $TAG done"
