set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r01_s3b
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r01_s3b/large.log 2>&1; rc=$?
tail -25 gpurun_out/r01_s3b/large.log; exit $rc
