set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r03}
# spec: world, frames per gather ("d": bench.py's default for the run length), steps, lead
for spec in "2 4 203 auto" "3 3 10 2" "2 2 9 4" "3 4 12 1" "2 8 20 auto" "2 d 20 auto" "3 d 45 1"; do
  set -- $spec
  K=""; [ "$2" = "d" ] || K="--frames-per-gather $2"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 \
      --master-port 29611 bench.py --gpus $1 --steps $3 --warmup 2 --spinup-frames 2 --no-cpu-baseline \
      --dist-backend gloo $K --rank0-lead $4 --lead-trial-frames 8 \
      > gpurun_out/dist_${TAG}_$1_$2_$4.json 2> gpurun_out/dist_${TAG}_$1_$2_$4.err
  rc=$?; echo "gloo rehearsal world=$1 K=$2 steps=$3 lead=$4 rc=$rc"; grep -h "frame-check" gpurun_out/dist_${TAG}_$1_$2_$4.err
  [ $rc -eq 0 ] || { tail -5 gpurun_out/dist_${TAG}_$1_$2_$4.err; exit $rc; }
done
