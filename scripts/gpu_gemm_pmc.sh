set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/pmc
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAVES --kernel-trace --output-format csv -d $R/gpurun_out/pmc/a -o g -- python3 $R/bench/gemm_one.py > $R/gpurun_out/pmc/a.log 2>&1 || { tail -20 $R/gpurun_out/pmc/a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc/b -o g -- python3 $R/bench/gemm_one.py > $R/gpurun_out/pmc/b.log 2>&1 || { tail -20 $R/gpurun_out/pmc/b.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc/c -o g -- python3 $R/bench/gemm_one.py > $R/gpurun_out/pmc/c.log 2>&1 || { tail -20 $R/gpurun_out/pmc/c.log; exit 1; }
ls -R $R/gpurun_out/pmc | head -30
