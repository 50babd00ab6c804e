# Round-4 check D (after C passed): persistent batch-1 decode A/B vs the per-kernel path, a
# rocprofv3 kernel-stats profile of one bench step, then the kernel GPU tests against the -DDA_DEBUG
# library (device asserts on; built beforehand in-tree: python -m docagents_amd.ops.build --debug).
# usage: bash scripts/gpu_r4d.sh TAG
set -u
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/${1:-r4d}; mkdir -p $OUT
timeout -k 10 300 python -u bench/b1_persistent_ab.py > $OUT/b1_persistent_ab.txt 2>&1
rc=$?; tail -4 $OUT/b1_persistent_ab.txt; [ $rc -ne 0 ] && exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o bench -- python3 $R/bench.py --steps 1 --warmup 1 --latency-reps 2 --ingest-docs 16 --breakdown 0 > $R/$OUT/prof_bench.json 2> $R/$OUT/prof_bench.err)
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/prof_bench.err; exit $rc; }
python bench/kstats_top.py $OUT/prof > $OUT/kstats_top.txt 2>&1; head -20 $OUT/kstats_top.txt
gzip -f $OUT/prof/*kernel_trace.csv
DA_KERNELS_DEBUG=1 timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_b1_gpu.py \
  tests/test_splitk_fused_gpu.py tests/test_fp16_encoder_gpu.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest_debug.log 2>&1
rc=$?; tail -4 $OUT/pytest_debug.log; exit $rc
