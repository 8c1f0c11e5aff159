set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && BENCH_DUMP_MERGES=/tmp/m.npy timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof -o run -- python3 $R/bench.py --no-encode --no-cpu > /tmp/b.log 2>&1
cd $R && EDGES=0,5,10,20,40,70,100,150,200,250,300,400,500,1000,2000,4000,8000,16000,24000 python tools/merge_profile.py /tmp/prof /tmp/m.npy > gpurun_out/mp_fine.txt 2>&1
python - > gpurun_out/spbits.txt <<'PY'
import csv,glob
rows=[]
for f in glob.glob('/tmp/prof/**/*kernel_trace.csv',recursive=True): rows+=list(csv.DictReader(open(f)))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
for r in rows:
    if 'k_sp_' in r['Kernel_Name'] or 'k_count_full' in r['Kernel_Name'] or 'fillBuffer' in r['Kernel_Name']:
        print(r['Kernel_Name'].split('(')[0][-40:], r.get('Grid_Size_X', r.get('Grid_Size','')), (int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
PY
tail -3 /tmp/b.log
