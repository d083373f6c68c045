# e2e (PCIe-inclusive) A/B of the sw_encode_batch pipeline: tests, then bench lines per variant.
set -u
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c3_split.py -k pipelined > gpurun_out/pipe_t.log 2>&1 || exit 1
for v in "$@"; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 4 $v > gpurun_out/e2e_ab_$(echo $v | tr -d ' -').log 2>&1 || exit 1
  echo "variant [$v]" >> gpurun_out/e2e_ab.txt
  grep '^{' gpurun_out/e2e_ab_$(echo $v | tr -d ' -').log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['e2e_pcie'])" >> gpurun_out/e2e_ab.txt
done
