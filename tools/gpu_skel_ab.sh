#!/bin/bash
# msda_bwd band-skeleton A/B (VS_MSDA_SKEL 0 vs the default 2): the MSDA parity tests, the kernel bench of both, then interleaved C2 bench runs.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/skel
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "msda or deform or train_parity" --timeout 200 --timeout-method thread > $O/tests_skel.log 2>&1
rc=$?; tail -2 $O/tests_skel.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/kbench.py --only msda --msda-modes skel0,prod,skel0,prod --iters 30 > $O/kbench.log 2>&1 || exit $?
grep msda $O/kbench.log
AB_A="VS_MSDA_SKEL=0" AB_B="VS_MSDA_SKEL=2" AB_ROUNDS=2 AB_STEPS=20 bash tools/ab.sh || exit $?
cat gpurun_out/ab/summary.txt
