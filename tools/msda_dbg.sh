# MSDA backward cost attribution (profiling builds only): VS_MSDA_WIN_DBG bits
#   1 skip the accumulation / walk / MFMA, 2 skip the per-cell atomics, 8 skip the
#   direct (clipped-corner) atomics, 16 skip the geom kernel, 32 skip the grad_value
#   kernel.  VS_MSDA_MFMA=1/0; VS_MSDA_BINNED: 4 / 8 (tile edge) or 0 (LDS-window walk)
cd ${GRAFT_REPO_ROOT:-.}
for cfg in ${CFGS:-"1 4" "0 4" "0 0"}; do
set -- $cfg
for d in ${DBGS:-0 1 2 8 16}; do
  echo "mfma=$1 binned=$2 dbg=$d $(VS_MSDA_MFMA=$1 VS_MSDA_BINNED=$2 VS_MSDA_WIN_DBG=$d timeout -k 10 120 python tools/kbench.py --only msda --iters 20 --msda-modes window | grep 'window.*msda_bwd' | tr '\n' ' ')"
done
done
