set -e
mkdir -p gpurun_out/reh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/reh/smoke.log 2>&1 || { tail -20 gpurun_out/reh/smoke.log; exit 1; }
tail -1 gpurun_out/reh/smoke.log
for w in mono_init tracking; do
  ORBGPU_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --workload $w --steps 20 --warmup 3 > gpurun_out/reh/rehearsal_$w.json 2> gpurun_out/reh/rehearsal_$w.err || { tail -20 gpurun_out/reh/rehearsal_$w.err; exit 1; }
  head -c 300 gpurun_out/reh/rehearsal_$w.json; echo
done
