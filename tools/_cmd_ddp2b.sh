# world-2 rehearsal on the 1-GPU box: the dist GPU tests, then bench.py under torchrun with
# gloo (RCCL refuses two ranks on one device) for cfg 2 and cfg 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -q --timeout 300 --timeout-method thread > gpurun_out/ddp_t.log 2>&1 || { tail -30 gpurun_out/ddp_t.log; exit 1; }
tail -1 gpurun_out/ddp_t.log
for c in 2 5; do
TTMI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951$c bench.py --gpus 2 --steps 20 --warmup 5 --config $c > gpurun_out/ddp2_gloo_c$c.log 2>&1 || { tail -30 gpurun_out/ddp2_gloo_c$c.log; exit 1; }
grep '"metric"' gpurun_out/ddp2_gloo_c$c.log | cut -c1-200
done
echo DONE
