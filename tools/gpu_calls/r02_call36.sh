# round 2: multi-rank rehearsal of the driver's scaling command on one GPU (2 ranks sharing it,
# gloo for the barrier / max / sum), with the IMIX leg and the host-side changes of this round
bash tools/gpu_session.sh \
 "rank2:400:UPE_BENCH_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/rank2.json"
