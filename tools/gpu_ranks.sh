# N=1 and N=2/4 (ranks sharing the box's one GPU) bench lines: the same HIP
# runtime at every rank count (bench.py's file rendezvous, no torch import)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/r1.json 2> gpurun_out/r1.err || { tail gpurun_out/r1.err; exit 1; }
for n in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/r$n.json 2> gpurun_out/r$n.err || { tail gpurun_out/r$n.err; exit 1; }
done
for n in 1 2 4; do python -c "import json;d=json.load(open('gpurun_out/r$n.json'));print($n, d['value'], d['ms_per_step'], d['parity']['ok'], d['hip_runtime'], d.get('e2e') and d['e2e'].get('verdicts_out'))"; done
