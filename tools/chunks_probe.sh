cd $GRAFT_REPO_ROOT
for k in 1 2 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-north-star --no-parity --no-entropy --chunks $k > gpurun_out/chunks_$k.json 2>gpurun_out/chunks_$k.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/chunks_$k.json'));print($k, d['value'], d['ms_per_step'], d['kernels_ms'])"
done
