set -o pipefail
bash benchmarks/gpu_lease.sh r3f tests smoke || exit $?
mkdir -p gpurun_out/r3f
timeout -k 10 400 python -u bench.py --gpus 4 --share-gpu --comm-backend gloo --steps 2 --warmup 2 --jobs 12 --out gpurun_out/r3f/share4.json > gpurun_out/r3f/share4.log 2>&1 || { tail -40 gpurun_out/r3f/share4.log; exit 5; }
tail -1 gpurun_out/r3f/share4.log | cut -c1-1500
