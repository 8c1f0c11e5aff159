# One GPU call of a session: the named steps in order, each under its own time
# limit, stopping at the first failure (tools/closing.sh is the round's final check).
#   tools/gpu_round.sh OUT STEP [STEP ...]
# STEP:
#   tests[=EXPR]        pytest -m gpu (-k EXPR)                 -> OUT/gpu_tests.txt
#   smoke               __graft_entry__.smoke()                 -> OUT/smoke.txt
#   bench[=ARGS]        python bench.py ARGS                     -> OUT/bench.json
#   'ab=LIBS -- NAMES'  tools/ab_libs.py LIBS -- NAMES (LIBS ' '-, NAMES ','-separated; AB_REPS / AB_ROUNDS
#                       from the environment)                    -> OUT/ab.txt
#   stats=ARGS          rocprofv3 --kernel-trace --stats over bench.py ARGS -> OUT/prof
#   c4=RANKS:SHARD      the C4 leg's self-check rehearsed with RANKS ranks sharing this one GPU over gloo
#                       (host-staged hand-over), SHARD bytes per rank -> OUT/c4_RANKSr_SHARD.json
#   'pmc=CTRS -- ARGS'  one rocprofv3 --pmc pass (CTRS ','-separated) over bench.py ARGS -> OUT/pmc_*
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p "$O"
L=gpu-bpe_amd/lib/libgpubpe.so
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=${step#*=}
  [ "$arg" = "$step" ] && arg=""
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$O/gpu_tests$n.txt" 2>&1 || { echo TESTFAIL; tail -40 "$O/gpu_tests$n.txt"; exit 1; }
      tail -1 "$O/gpu_tests$n.txt" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1 \
        || { echo SMOKEFAIL; tail -20 "$O/smoke.txt"; exit 1; }
      tail -1 "$O/smoke.txt" ;;
    bench)
      timeout -k 10 900 python bench.py $arg > "$O/bench$n.json" 2> "$O/bench$n.err" \
        || { echo BENCHFAIL; tail -20 "$O/bench$n.err"; exit 1; }
      tail -c 1500 "$O/bench$n.json" ;;
    ab)
      libs=${arg%% -- *}
      names=${arg#* -- }
      timeout -k 10 1000 python -u tools/ab_libs.py $libs -- ${names//,/ } > "$O/ab$n.txt" 2>&1 \
        || { echo ABFAIL; tail -30 "$O/ab$n.txt"; exit 1; }
      grep -E "min [0-9.]+ s" "$O/ab$n.txt"
      grep -o '"paired": [0-9]*' "$O/ab$n.txt" | sort | uniq -c | head -5 ;;
    stats)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof$n" -o run -- python3 bench.py $arg \
        > "$O/stats$n.json" 2> "$O/stats$n.err" || { echo STATSFAIL; tail -20 "$O/stats$n.err"; exit 1; }
      find "$O/prof$n" -name "*kernel_stats.csv" | head -1 | xargs -r head -12 ;;
    pmc)
      ctrs=${arg%% -- *}
      args=${arg#* -- }
      timeout -s KILL 300 rocprofv3 --pmc ${ctrs//,/ } -d "$O/pmc$n" -o run -- python3 bench.py $args \
        > "$O/pmc$n.json" 2> "$O/pmc$n.err" || { echo PMCFAIL; tail -20 "$O/pmc$n.err"; exit 1; }
      echo "pmc$n done" ;;
    c4)
      rk=${arg%%:*}
      sh=${arg#*:}
      GBPE_BENCH_DEVICE=0 GBPE_SHARD_TRANSPORT=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $rk --master-addr 127.0.0.1 --master-port 29574 bench.py --gpus $rk --c4-only --c4-shard $sh \
        > "$O/c4_${rk}r_$sh.json" 2> "$O/c4_${rk}r_$sh.err" || { echo C4FAIL; tail -30 "$O/c4_${rk}r_$sh.err"; exit 1; }
      python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);c=d['c4'];print('c4',c['value'],c.get('counts_equal_recount'),c['timing_s_max_over_ranks'])" "$O/c4_${rk}r_$sh.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
