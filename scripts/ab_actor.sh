bash scripts/gpu.sh "tests:actor or full_pool or bf16x6 or mopo" || exit 1
: > gpurun_out/actor_ab.txt
for i in 1 2; do
  for act in bf16x6 fp32; do
    timeout -k 10 150 python bench.py --no-cpu-baseline --no-c3 --no-alt-dtypes --train-epochs 0 --sac-steps 16 --actor-dtype $act > gpurun_out/aab.json 2>gpurun_out/aab.err || { tail -5 gpurun_out/aab.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/aab.json').read().strip().splitlines()[-1]); k=d['kernel_ms_avg']; print('$act', round(d['value']/1e6,2), 'M/s ens', k['ensemble_fwd'], 'actor', k['actor'])" >> gpurun_out/actor_ab.txt
  done
done
cat gpurun_out/actor_ab.txt
