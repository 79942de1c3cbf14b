set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/p1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/eager -o bench -- python3 bench.py --no-cpu-baseline --no-parity --graphs 0 --steps 3 --warmup 2 > $O/eager.log 2>&1 || exit $?
f=$(ls $O/eager/*/bench_kernel_trace.csv $O/eager/bench_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/step_breakdown.py $f 60 > $O/breakdown.txt || exit $?
echo done
