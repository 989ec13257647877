# Disentangled-attention timing + SQ counters at the cfg-4 shape (tools/attn_bench.py).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 -u $R/tools/attn_bench.py > $R/gpurun_out/dis_time.log 2>&1 || { tail -20 $R/gpurun_out/dis_time.log; exit 1; }
cat $R/gpurun_out/dis_time.log
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/dis_pmc$i -o run -- python3 $R/tools/attn_bench.py > $R/gpurun_out/dis_pmc$i.log 2>&1 || { tail -20 $R/gpurun_out/dis_pmc$i.log; exit 1; }
done
python3 $R/tools/pmc_kernels.py dis_ $(ls $R/gpurun_out/dis_pmc*/*/run_counter_collection.csv $R/gpurun_out/dis_pmc*/run_counter_collection.csv 2>/dev/null)
echo DONE
