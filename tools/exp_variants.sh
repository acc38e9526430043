set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
V=ggml-neon-opt_amd/lib/variants
timeout -k 10 600 python tools/gemv_sweep.py auto lib=$V/libw8.so lib=$V/libw16.so lib=$V/libw12d4.so > gpurun_out/sweep5.log 2>&1 || exit $?
for L in "" $V/libw8.so $V/libw16.so $V/libw12d4.so; do
  if [ -n "$L" ]; then export MI355X_LIB=$PWD/$L; else unset MI355X_LIB; fi
  echo "lib=${L:-default}" >> gpurun_out/bench5.log
  timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-large 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernels'])" >> gpurun_out/bench5.log || exit $?
done
cat gpurun_out/sweep5.log gpurun_out/bench5.log
