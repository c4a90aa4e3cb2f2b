#!/bin/bash
# Round 4 (z): the C++ frame loop (examples/frame_loop.cpp, the reference's
# frame with the disk update on a side stream) on each library given,
# interleaved, 3 repetitions; every library's frames must equal the first's.
#   bash tools/gpu_r04z.sh A.so B.so [C.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04z
mkdir -p $OUT
LIB=schwarzschild_raytracer_wgpu_amd/libgeo.so
LIBS=("$@")
cp "$LIB" $OUT/.orig.so
g++ -std=c++17 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include examples/frame_loop.cpp \
    -L schwarzschild_raytracer_wgpu_amd -lgeo -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$(pwd)/schwarzschild_raytracer_wgpu_amd \
    -Wl,-rpath,/opt/rocm/lib -o $OUT/frame_loop || exit 1
: > $OUT/frame_loop_ab.txt
for rep in 1 2 3; do
  i=0
  for v in "${LIBS[@]}"; do
    cp "$v" "$LIB"
    for run in "1920 1080 3000 fan" "3840 2160 2000 fan" "1920 1080 2000 direct"; do
      set -- $run
      M=""; [ "$4" = fan ] && M=fan
      line=$(timeout -k 10 120 $OUT/frame_loop $1 $2 $3 $OUT/f_${i}_$2_$4.ppm 1 $M) || { cp $OUT/.orig.so "$LIB"; exit 1; }
      echo "$(basename $v) rep$rep: $line" | tee -a $OUT/frame_loop_ab.txt
      if [ $i -gt 0 ]; then cmp $OUT/f_0_$2_$4.ppm $OUT/f_${i}_$2_$4.ppm || { echo "frames differ"; cp $OUT/.orig.so "$LIB"; exit 1; }; fi
    done
    i=$((i + 1))
  done
done
cp $OUT/.orig.so "$LIB"
rm -f $OUT/*.ppm
echo "frames equal across libraries"
