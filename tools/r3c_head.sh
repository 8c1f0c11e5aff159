set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
# Round-3 re-entry check at HEAD: the GPU suite, smoke and the default bench line.
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/gpu_tests.txt 2>&1
tail -2 gpurun_out/r3c/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3c/smoke.txt 2>&1
tail -1 gpurun_out/r3c/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r3c/bench.json 2> gpurun_out/r3c/bench.err
tail -c 400 gpurun_out/r3c/bench.json
# then: per-merge kernel profile of one 1 GiB headline run at HEAD (merges bucketed by index) and the
# kernel timeline of its first launches.
mkdir -p $R/gpurun_out/r3c
python -c "import numpy as np; np.save('/tmp/m.npy', np.load('$R/tests/golden/train_en1g.npz')['merges'])"
cd /tmp && EXPLORE_REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof -o run -- python3 $R/tools/explore_1g.py en1g > /tmp/b.log 2>&1
cd $R && EDGES=0,10,50,100,200,300,500,1000,2000,4000,8000,16000,24000 python tools/merge_profile.py /tmp/prof /tmp/m.npy > gpurun_out/r3c/merge_profile_en1g.txt 2>&1
python tools/trace_timeline.py /tmp/prof 600 > gpurun_out/r3c/timeline_en1g.txt 2>&1
tail -2 /tmp/b.log
