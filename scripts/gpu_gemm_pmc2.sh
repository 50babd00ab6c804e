# PMC counters (SQ wait/busy, MFMA busy, LDS) for the 8-wave (tile 4) and 4-wave (tile 5) 256x256 GEMMs.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/pmc2
python -m docagents_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 3; }
cd /tmp && export TMPDIR=/tmp
for T in 4 5; do
  export TILE=$T
  timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $R/gpurun_out/pmc2/b$T -o g -- python3 $R/bench/gemm_one.py > $R/gpurun_out/pmc2/b$T.log 2>&1 || { tail -20 $R/gpurun_out/pmc2/b$T.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc2/c$T -o g -- python3 $R/bench/gemm_one.py > $R/gpurun_out/pmc2/c$T.log 2>&1 || { tail -20 $R/gpurun_out/pmc2/c$T.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $R/gpurun_out/pmc2/d$T -o g -- python3 $R/bench/gemm_one.py > $R/gpurun_out/pmc2/d$T.log 2>&1 || { tail -20 $R/gpurun_out/pmc2/d$T.log; exit 1; }
done
echo done
