# split-K weight-gradient tile target A/B (VS_SPLITK_TILES) on the C5 and C2 bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for t in 768 1536 3072; do
  VS_SPLITK_TILES=$t timeout -k 10 300 python3 bench.py --model swin_l --size 1536 --no-cpu-baseline --no-parity --steps 5 > gpurun_out/sk_c5_$t.log 2>&1 || exit $?
  echo "C5 tiles $t: $(tail -1 gpurun_out/sk_c5_$t.log | cut -c80-140)"
done
for t in 768 1536; do
  VS_SPLITK_TILES=$t timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-parity > gpurun_out/sk_c2_$t.log 2>&1 || exit $?
  echo "C2 tiles $t: $(tail -1 gpurun_out/sk_c2_$t.log | cut -c80-140)"
done
