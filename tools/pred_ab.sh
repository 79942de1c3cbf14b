cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
M=vision-instance-seg_amd/visionseg/model.py
for i in 1 2; do timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -k predictor tests/test_gpu_model.py > gpurun_out/pred_new_$i.log 2>&1; echo "new $i rc=$?"; done
cp gpurun_model_old.py $M || exit 1
for i in 1 2; do timeout -k 10 200 python -u -m pytest -q --timeout 150 --timeout-method thread -k predictor tests/test_gpu_model.py > gpurun_out/pred_old_$i.log 2>&1; echo "old $i rc=$?"; done
