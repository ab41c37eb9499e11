#!/bin/bash
# One parameterised runner for gpurun calls (replaces the old one-off scripts).
#
#   gpurun --timeout 900 -- bash scripts/gpu_job.sh TAG job [job ...]
#
# Every job runs under its own time limit; the call stops at the first crash,
# timeout or GPU-fault message. Logs land in gpurun_out/TAG_<job>.txt.
#
# jobs:
#   tests            pytest -m gpu (whole GPU suite)
#   tests:EXPR       pytest -m gpu -k EXPR   (commas become spaces: tests:a,or,b)
#   testss:EXPR      the same with -s and a 600 s per-test limit (long numerics tests)
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     python bench.py ARGS   (ARGS: commas become spaces)
#   benchenv:K=V+K2=V2[:ARGS]  the same with extra environment variables
#   ktrace[:ARGS]    rocprofv3 kernel trace of bench.py --steps 3 --warmup 3 ARGS,
#                    per-step summary via scripts/step_profile.py
#   hiptrace[:ARGS]  rocprofv3 HIP-API + kernel trace (host-sync hunting)
#   pmc:CTRS:ARGS    one counter pass (CTRS: commas -> spaces) over bench.py ARGS
#   pmcpy:CTRS:SCRIPT[:ARGS]  one counter pass over python3 SCRIPT ARGS
#   py:SCRIPT[:ARGS] python SCRIPT ARGS
#   pyenv:K=V+K2=V2:SCRIPT[:ARGS]  the same with extra environment variables
#   retunewith:NAME:IDS[:ARGS]  targeted re-tune of the shipped conv_nt keys against ids IDS
#                    (e.g. 45-48+50: '+' separates ranges) -> gpurun_out/tune_NAME.json
source "$(dirname "$0")/gpurun_lib.sh"
TAG=$1; shift
for job in "$@"; do
  name=${job%%:*}; rest=""; [[ "$job" == *:* ]] && rest=${job#*:}
  args=${rest//,/ }
  case $name in
    tests)
      if [ -n "$rest" ]; then
        run ${TAG}_tests_$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-40).txt 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$args"
      else
        run ${TAG}_tests.txt 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
      fi ;;
    testss)  # like tests:EXPR but with -s (prints stream into the log: long tests show progress)
      PDT_SLOW_TESTS=1 run ${TAG}_testss_$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-40).txt 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread -k "$args" ;;
    smoke) run ${TAG}_smoke.txt 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run ${TAG}_bench_$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_').txt 400 python bench.py $args ;;
    benchenv)  # benchenv:K=V+K2=V2:ARGS -- bench.py with extra environment variables
      envs=${rest%%:*}; bargs=""; [[ "$rest" == *:* ]] && bargs=${rest#*:}
      run ${TAG}_benchenv_$(echo "$envs$bargs" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-60).txt 400 env ${envs//+/ } python bench.py ${bargs//,/ } ;;
    benchlong)  # stock-stack runs whose MIOpen find takes minutes; find results kept in gpurun_out/miopen_db,
                # seeded from the find db of earlier runs (profiles/miopen_db_bs2048: MIOpen's own text db)
      mkdir -p gpurun_out/miopen_db
      cp -n profiles/miopen_db_bs2048/*.txt gpurun_out/miopen_db/ 2>/dev/null || true
      export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
      run ${TAG}_benchlong_$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_').txt 1000 python bench.py $args ;;
    ktrace)
      sfx=$(echo "$args" | tr -c 'a-zA-Z0-9_\n' '_')
      d=gpurun_out/${TAG}_ktrace$sfx
      run ${TAG}_ktrace$sfx.txt 400 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 3 $args
      f=$(find $d -name '*kernel_trace.csv' | head -n 1)
      python scripts/step_profile.py "$f" --top 60 > gpurun_out/${TAG}_ktrace${sfx}_step.txt 2>&1 || true ;;
    hiptrace)
      d=gpurun_out/${TAG}_hiptrace
      run ${TAG}_hiptrace.txt 400 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 3 $args ;;
    pmc)
      ctrs=${rest%%:*}; bargs=""; [[ "$rest" == *:* ]] && bargs=${rest#*:}
      sfx=$(echo "$ctrs$bargs" | md5sum | cut -c1-8)  # (counters + bench args: one directory per pass)
      d=gpurun_out/${TAG}_pmc_$sfx
      run ${TAG}_pmc_$sfx.txt 240 timeout -s KILL 200 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d $d -o run -- python3 bench.py --steps 2 --warmup 2 ${bargs//,/ } ;;
    pmcpy)  # pmcpy:CTRS:SCRIPT[:ARGS] -- one counter pass over a python script
      ctrs=${rest%%:*}; r2=${rest#*:}; scr=${r2%%:*}; sargs=""; [[ "$r2" == *:* ]] && sargs=${r2#*:}
      sfx=$(echo "$ctrs$scr$sargs" | md5sum | cut -c1-8)
      d=gpurun_out/${TAG}_pmc_$sfx
      run ${TAG}_pmc_$sfx.txt 240 timeout -s KILL 200 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d $d -o run -- python3 -u $scr ${sargs//,/ } ;;
    retune)  # fresh autotune of every kernel variant for a bench config -> gpurun_out/tune_NAME.json
      nm=${rest%%:*}; bargs=""; [[ "$rest" == *:* ]] && bargs=${rest#*:}
      PDT_AUTOTUNE_SHIPPED=0 PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_$nm.json run ${TAG}_retune_$nm.txt 600 python bench.py --steps 5 --warmup 3 ${bargs//,/ } ;;
    retunewith)  # targeted re-tune: every shipped conv_nt key vs the ids IDS only -> gpurun_out/tune_NAME.json
      nm=${rest%%:*}; r2=${rest#*:}; ids=${r2%%:*}; bargs=""; [[ "$r2" == *:* ]] && bargs=${r2#*:}
      PDT_TUNE_ROUNDS=4 PDT_RETUNE_WITH=${ids//+/,} PDT_RETUNE_AX=${PDT_RETUNE_AX//+/,} PDT_AUTOTUNE_CACHE=$PWD/gpurun_out/tune_$nm.json run ${TAG}_retunewith_$nm.txt 600 python bench.py --steps 5 --warmup 3 ${bargs//,/ } ;;
    py)
      scr=${rest%%:*}; sargs=""; [[ "$rest" == *:* ]] && sargs=${rest#*:}
      run ${TAG}_py_$(basename $scr .py)$(echo "$sargs" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-30).txt 600 python -u $scr ${sargs//,/ } ;;
    pyenv)  # pyenv:K=V+K2=V2:SCRIPT[:ARGS] -- a python script with extra environment variables
      envs=${rest%%:*}; r2=${rest#*:}; scr=${r2%%:*}; sargs=""; [[ "$r2" == *:* ]] && sargs=${r2#*:}
      run ${TAG}_pyenv_$(echo "$envs$(basename $scr .py)$sargs" | tr -c 'a-zA-Z0-9_\n' '_' | cut -c1-60).txt 600 env ${envs//+/ } python -u $scr ${sargs//,/ } ;;
    *) echo "unknown job $job"; exit 2 ;;
  esac
done
exit 0
