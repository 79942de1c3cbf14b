cd /tmp && export TMPDIR=/tmp
for e in ${MH_EXPS:-0 1 2 3 8 9 11}; do
  VS_MH_EXP=$e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/mhx$e -o run -- python3 /root/repo/tools/kbench.py --only mask --iters 10 > /root/repo/gpurun_out/mhx$e.log 2>&1 || exit 1
done
