# LayerNorm backward A/B: the kernel's own time per Swin stage shape (rocprofv3 kernel
# trace of tools/lnbench.py at the default workgroup cap), current library vs the one in
# gpurun_ab_old.so (built from the previous source), after the op tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -k "layer_norm or column_sum or activation_backward" tests/test_gpu_ops.py > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
tail -1 gpurun_out/ln_tests.log
L=vision-instance-seg_amd/visionseg/libvisionseg_hip.so
for v in new old; do
  if [ $v = old ]; then cp $L /tmp/lib_new.so && cp gpurun_ab_old.so $L || exit 1; fi
  LNB_PARTS=512 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lnprof_$v -o ln -- python3 tools/lnbench.py > gpurun_out/lnbench_$v.txt 2>&1 || exit $?
  python3 - $v <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(f"gpurun_out/lnprof_{sys.argv[1]}/ln_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
shapes = ["M 262144 C 96", "M 65536 C 192", "M 589824 C 192", "M 147456 C 384"]
for kname, per in (("ln_bwd", 23), ("ln_fwd", 24)):
    t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if kname in r["Kernel_Name"]]
    for i, sh in enumerate(shapes):
        g = t[per * i + per - 20: per * i + per]
        print(f"{sys.argv[1]} {sh}: {kname}_kernel mean {sum(g) / max(1, len(g)):.1f} us over {len(g)}")
PY
  rm -rf gpurun_out/lnprof_$v
done
cp /tmp/lib_new.so $L
