cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python tools/fp8_debug.py > gpurun_out/r3_fp8_debug.txt 2>&1; cat gpurun_out/r3_fp8_debug.txt | grep -v "sample"
