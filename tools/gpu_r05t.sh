set -u
O=gpurun_out/r05t
mkdir -p $O
b() { timeout -k 10 300 "$@" --no-cpu-baseline; }
timeout -k 10 600 python -u -m pytest tests/test_golden_scale.py -k "c3nl" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_c3nl.log 2>&1 &&
b python bench.py --workload c3nl --steps 1000 > $O/c3nl_1000.json 2> $O/e1 &&
b python bench.py --workload c3nl --steps 200 > $O/c3nl_200.json 2> $O/e2 &&
b python bench.py --steps 1000 > $O/c3.json 2> $O/e3 &&
b python bench.py --workload c4 --steps 1000 > $O/c4.json 2> $O/e4 &&
timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > $O/sh_fused.json 2> $O/e7 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
