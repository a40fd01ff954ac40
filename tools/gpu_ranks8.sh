# configs[3] rehearsal on one GPU: 8 ranks x 2^24 packets = 128M packets
# through bench.py's file rendezvous and host merge (the driver's N=8 run
# uses 8 GPUs; here the ranks share the box's one GPU, so the rate is the
# one GPU's, and what is checked is the 8-shard merge: parity.ok and the
# merged counter = 8 x 2^24 x 23)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 10 --warmup 3 > gpurun_out/r8.json 2> gpurun_out/r8.err || { tail -30 gpurun_out/r8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r8.json'));print(8, d['value'], d['ms_per_step'], d['parity'], d['config'].get('packets_per_gpu'))"
