# which earlier test of tests/test_gpu_model.py breaks the Predictor graph test (debug aid)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for k in "train_template_seam and maskdino or predictor" "tiny_model or predictor" "not predictor or predictor"; do
  timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -k "$k" tests/test_gpu_model.py > gpurun_out/bis.log 2>&1
  echo "[$k] rc=$? $(tail -1 gpurun_out/bis.log)"
done
