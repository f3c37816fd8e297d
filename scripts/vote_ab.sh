# Hough op time at B = 1, 2, 4, 8 (run through gpurun; the vote geometry A/B of round 3 used it with a temporary PCNN_VOTE_CFG override)
: > gpurun_out/vote_ab.log
for i in 1 2; do
for c in tree; do
  echo "== $c" >> gpurun_out/vote_ab.log
  for b in 1 2 4 8; do
    t=""; [ $b = 1 ] && t="--test"
    timeout -k 10 120 python scripts/hough_bench.py --batch $b $t --iters 100 >> gpurun_out/vote_ab.log 2>&1 || exit 1
  done
done
done
