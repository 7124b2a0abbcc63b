set -o pipefail
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --out gpurun_out/ab_ev$i.json > /dev/null 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-kernel-events --out gpurun_out/ab_noev$i.json > /dev/null 2>&1 || exit $?
done
echo done
