set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TTMI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/ddp2_gloo.log 2>&1 || { tail -30 gpurun_out/ddp2_gloo.log; exit 1; }
grep '"metric"' gpurun_out/ddp2_gloo.log | cut -c1-260
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/ddp2_nccl.log 2>&1; echo "nccl rc=$?"; grep -E '"metric"|Error|error' gpurun_out/ddp2_nccl.log | head -5 | cut -c1-300
echo DONE
