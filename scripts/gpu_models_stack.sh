# Model GPU tests (incl. prompt-head cache under graphs), then the full HTTP stack loadgen.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_models.log 2>&1 || { tail -30 gpurun_out/t_models.log; exit 1; }
tail -1 gpurun_out/t_models.log
bash scripts/gpu_stack.sh
