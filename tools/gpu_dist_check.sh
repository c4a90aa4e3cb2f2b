#!/bin/bash
# One GPU box: GPU tests, the default bench, host-overhead probe, and 2- and
# 3-rank gloo rehearsals of the multi-GPU frame loop on the one GPU (batched
# gathers, partial last batch, plain and lead layouts, the lead auto-trial)
# with the assembled frame checked.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu_$TAG.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$TAG.err; exit $rc; }
timeout -k 10 200 python tools/host_overhead.py > gpurun_out/host_overhead_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/host_overhead_$TAG.log; [ $rc -eq 0 ] || exit $rc
for spec in "2 4 203 auto" "3 3 10 2" "2 2 9 4" "3 4 12 1"; do
  set -- $spec
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
      --master-port 29611 bench.py --gpus $1 --steps $3 --warmup 2 --spinup-frames 2 --no-cpu-baseline \
      --dist-backend gloo --frames-per-gather $2 --rank0-lead $4 --lead-trial-frames 8 \
      > gpurun_out/dist_${TAG}_$1_$4.json 2> gpurun_out/dist_${TAG}_$1_$4.err
  rc=$?; echo "gloo rehearsal world=$1 K=$2 steps=$3 lead=$4 rc=$rc"; grep -h "frame-check" gpurun_out/dist_${TAG}_$1_$4.err
  [ $rc -eq 0 ] || { tail -5 gpurun_out/dist_${TAG}_$1_$4.err; exit $rc; }
done
