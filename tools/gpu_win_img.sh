# image-layout window attention: op tests (new equality test + existing window / fp8), then
# model tests (Swin through window_attention_image) and the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -k "window or fp8 or layer_norm" tests/test_gpu_ops.py tests/test_gpu_fp8.py > gpurun_out/win_img.log 2>&1 || { tail -30 gpurun_out/win_img.log; exit 1; }
tail -1 gpurun_out/win_img.log
bash tools/gpu_model_check.sh
