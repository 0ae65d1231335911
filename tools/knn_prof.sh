set -e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/knnprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/knn_probe.py --q 1024 > $GRAFT_REPO_ROOT/gpurun_out/knnprof/out.txt 2>&1
cat $GRAFT_REPO_ROOT/gpurun_out/knnprof/out.txt | grep search
