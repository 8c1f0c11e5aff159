# The round's profiles of the bench workloads (one GPU call; every step under its own
# time limit, outputs under gpurun_out/$OUT, default "prof"):
#   stats   rocprofv3 --kernel-trace --stats of one full en1g run     -> en1g_kernel_stats.csv
#   kbody   two --pmc passes (FETCH_SIZE, WRITE_SIZE) of one en1g run -> pmc_kbody.json
#   encode  kernel trace + two --pmc passes of one C3 encode          -> c3_encode_kernel_stats.csv, pmc_encode.json
#   walk    the encode walk's cache / stall counters                  -> pmc_walk.txt
#   sq=CORPUS[:STEPS]  k_body wave-cycle split (SQ counters) over the first STEPS steps of CORPUS
#   tools/profile_round.sh stats kbody encode        (then copy what is judged to profiles/rN/)
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/${OUT:-prof}
mkdir -p $O
cd /tmp
for step in "$@"; do
  case ${step%%=*} in
    stats)
      rm -rf /tmp/ks
      EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ks -o run -- \
        python3 $R/tools/explore_1g.py ${WL:-en1g} > $O/ks.log 2>&1 || { echo STATSFAIL; tail $O/ks.log; exit 1; }
      cp $(find /tmp/ks -name "*kernel_stats.csv") $O/${WL:-en1g}_kernel_stats.csv
      head -8 $O/${WL:-en1g}_kernel_stats.csv | cut -c1-160 ;;
    kbody)
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf /tmp/p$c
        EXPLORE_REPS=1 timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d /tmp/p$c -o run -- \
          python3 $R/tools/explore_1g.py en1g > $O/p$c.log 2>&1 || { echo PMCFAIL $c; tail $O/p$c.log; exit 1; }
      done
      python3 $R/tools/pmc_r2.py kbody /tmp/pFETCH_SIZE /tmp/pWRITE_SIZE $O/pFETCH_SIZE.log $O/pmc_kbody.json && cat $O/pmc_kbody.json ;;
    encode)
      rm -rf /tmp/eks
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/eks -o run -- \
        python3 $R/tools/encode_once.py 3 > $O/eks.log 2>&1 || { echo ENCSTATSFAIL; tail $O/eks.log; exit 1; }
      cp $(find /tmp/eks -name "*kernel_stats.csv") $O/c3_encode_kernel_stats.csv
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf /tmp/e$c
        timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d /tmp/e$c -o run -- \
          python3 $R/tools/encode_once.py 3 > $O/e$c.log 2>&1 || { echo ENCPMCFAIL $c; tail $O/e$c.log; exit 1; }
      done
      python3 $R/tools/pmc_r2.py encode /tmp/eFETCH_SIZE /tmp/eWRITE_SIZE $O/eFETCH_SIZE.log $O/pmc_encode.json && cat $O/pmc_encode.json ;;
    walk)
      i=0
      for set in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
                 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY"; do
        i=$((i + 1))
        timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d /tmp/pw$i -o run -- \
          python3 $R/tools/encode_once.py 1 > $O/pw$i.log 2>&1 || { echo WALKFAIL $i; tail $O/pw$i.log; exit 1; }
        python3 $R/tools/pmc_kernel_sum.py /tmp/pw$i walk >> $O/pmc_walk.txt
      done
      cat $O/pmc_walk.txt ;;
    sq)
      a=${step#*=}
      c=${a%%:*}
      n=${a#*:}; [ "$n" = "$a" ] && n=4
      EXPLORE_REPS=1 EXPLORE_MAX_STEPS=$n timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d /tmp/sq \
        -o run -- python3 $R/tools/explore_1g.py $c > $O/sq.log 2>&1 || { echo SQFAIL; tail $O/sq.log; exit 1; }
      python3 $R/tools/pmc_kernel_sum.py /tmp/sq "k_body<" > $O/pmc_sq_$c.txt && cat $O/pmc_sq_$c.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
