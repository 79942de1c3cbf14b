#!/bin/bash
# msda column kernel (tests, kernel bench, PMC traffic), then the token GEMM + window XCD A/B
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r4_msda.sh; rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/r4_msda_pmc.sh || exit $?
bash tools/r4_tgemm.sh
