# Per-merge kernel profile of one full 1 GiB English run (en1g) plus the PMC
# traffic passes the bench line cites (one GPU call):
#   1. rocprofv3 --kernel-trace over tools/explore_1g.py en1g -> gpurun_out/mp_en1g.txt
#   2. FETCH_SIZE / WRITE_SIZE passes over the same run        -> gpurun_out/r2_pmc_kbody.json
#   3. FETCH_SIZE / WRITE_SIZE passes over one C3 encode       -> gpurun_out/r2_pmc_encode.json
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C=${1:-en1g}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt1g -o run -- python3 $R/tools/explore_1g.py $C > /tmp/kt1g.log 2>&1
cp /tmp/kt1g.log $R/gpurun_out/kt1g_$C.log
cd $R && EDGES=0,10,50,100,128,150,200,300,500,1000,2000,4000,8000,16000,24000 python3 tools/merge_profile.py /tmp/kt1g gpurun_out/explore_${C}_merges.npy > gpurun_out/mp_$C.txt 2>&1
[ -n "$SKIP_PMC" ] && exit 0
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pf.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/pw.log 2>&1
python3 $R/tools/pmc_r2.py kbody /tmp/pf /tmp/pw /tmp/pf.log $R/gpurun_out/r2_pmc_kbody.json
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ef -o run -- python3 $R/tools/encode_once.py 2 > /tmp/ef.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/ew -o run -- python3 $R/tools/encode_once.py 2 > /tmp/ew.log 2>&1
python3 $R/tools/pmc_r2.py encode /tmp/ef /tmp/ew /tmp/ef.log $R/gpurun_out/r2_pmc_encode.json
