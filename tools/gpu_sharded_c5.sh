cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-sh2}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 -- python3 -u bench.py --sharded --workload c5 --steps 6 --warmup 2 > $O/c5.json 2> $O/c5.err
echo rc=$?; cat $O/c5.json; f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -20
