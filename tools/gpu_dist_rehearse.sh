#!/bin/bash
# gloo rehearsals of the multi-rank present path on one GPU (world 2 and 3,
# both launchers, several gather batch sizes and rank-0 leads): every run's
# frame_check must pass.  The driver's N = 8 form is tools/evidence.sh gloo8.
#   TAG=r05 bash tools/gpu_dist_rehearse.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
# spec: world, frames per gather ("d": bench.py's default for the run length), steps, lead, launcher
# (torchrun, or "self": bench.py starts its own ranks)
for spec in "2 4 203 auto torchrun" "3 3 10 2 self" "2 2 9 4 self" "3 4 12 1 torchrun" "2 8 20 auto self" \
            "2 d 20 auto self" "3 d 45 1 self"; do
  set -- $spec
  K=""; [ "$2" = "d" ] || K="--frames-per-gather $2"
  if [ "$5" = "self" ]; then LAUNCH="python"; else
    LAUNCH="python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 29611"; fi
  timeout -k 10 300 $LAUNCH bench.py --gpus $1 --steps $3 --warmup 2 --spinup-frames 2 --no-cpu-baseline \
      --dist-backend gloo $K --rank0-lead $4 --lead-trial-frames 8 \
      > gpurun_out/dist_${TAG}_$1_$2_$4.json 2> gpurun_out/dist_${TAG}_$1_$2_$4.err
  rc=$?; echo "gloo rehearsal world=$1 K=$2 steps=$3 lead=$4 launcher=$5 rc=$rc"; grep -h "frame-check" gpurun_out/dist_${TAG}_$1_$2_$4.err
  [ $rc -eq 0 ] || { tail -5 gpurun_out/dist_${TAG}_$1_$2_$4.err; exit $rc; }
done
