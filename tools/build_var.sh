# A library variant for A/B runs: one kernel unit rebuilt with extra hipcc
# flags, every other object from the in-tree build (make first), into
# gpurun_var/<name>/lib.so (travels to the box; git-ignored; loaded through
# GIC_LIBRARY=gpurun_var/<name>/lib.so).
#   bash tools/build_var.sh NAME UNIT [extra hipcc flags]    UNIT: gic_bcx | gic_bc7 | gic_bc7enc | gic_bc6h
set -e
NAME=$1; UNIT=$2; shift 2
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
cd $D
T=$(mktemp -d)
/opt/rocm/bin/hipcc $F "$@" -c csrc/$UNIT.hip -o $T/$UNIT.o
OBJS=""
for u in gic_bcx gic_bc7 gic_bc7enc gic_bc6h gic_api gic_multi gic_pipeline; do
  if [ $u = $UNIT ]; then OBJS="$OBJS $T/$u.o"; else OBJS="$OBJS build/$u.o"; fi
done
mkdir -p ../gpurun_var/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_var/$NAME/lib.so $OBJS -L/opt/rocm/lib -lrccl -lpthread
rm -rf $T
echo built $NAME
