#!/bin/bash
# Round-2 measurement session after the LDS-chain folds: bench lines (+ the incremental mode) (driver flags and long runs) for c3/c2/c4/c5,
# rocprofv3 kernel-trace summaries of c3 and c5, PMC FETCH/WRITE passes for c5.
# Every GPU step has its own time limit; the script stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02e
O=gpurun_out/r02e
run() { local name=$1 lim=$2; shift 2; echo "== $name: $*" >> $O/log.txt; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ] || { tail -20 $O/$name.out >> $O/log.txt; exit $rc; }; }
run c3_driver 300 python3 -u bench.py --steps 20 --warmup 5
run c3_1000 300 python3 -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline
run c2 300 python3 -u bench.py --workload c2 --steps 100 --warmup 0 --no-cpu-baseline
run c4 300 python3 -u bench.py --workload c4 --steps 1000 --warmup 0 --no-cpu-baseline
run c5 400 python3 -u bench.py --workload c5 --steps 200 --warmup 5 --no-cpu-baseline
run c3_incr 300 python3 -u bench.py --mode incremental --steps 1000 --warmup 20 --no-cpu-baseline
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline
run prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --steps 200 --warmup 5 --no-cpu-baseline
run pmc_c3_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmcc3_FETCH_SIZE -o run -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline
run pmc_c3_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmcc3_WRITE_SIZE -o run -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline
run pmc_c5_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmcc5_FETCH_SIZE -o run -- python3 bench.py --workload c5 --steps 100 --warmup 5 --no-cpu-baseline
run pmc_c5_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmcc5_WRITE_SIZE -o run -- python3 bench.py --workload c5 --steps 100 --warmup 5 --no-cpu-baseline
echo ALLDONE >> $O/log.txt
