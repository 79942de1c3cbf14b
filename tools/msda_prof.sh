set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for d in 0 1 2 3; do VS_MSDA_WG=0 VS_MSDA_WIN_DBG=$d timeout -k 10 120 python tools/kbench.py --only msda --iters 20 > gpurun_out/kb_dbg$d.txt; done
VS_MSDA_WG=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wg0 -o run -- python tools/kbench.py --only msda --iters 10 > /dev/null
VS_MSDA_WG=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wg1 -o run -- python tools/kbench.py --only msda --iters 10 > /dev/null
