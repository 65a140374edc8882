# A library variant for A/B runs: one kernel unit rebuilt with extra hipcc
# flags, every other object from the in-tree build (make first), into
# gpurun_var/<name>/lib.so (travels to the box; git-ignored; loaded through
# GIC_LIBRARY=gpurun_var/<name>/lib.so).
#   bash tools/build_var.sh NAME UNIT [extra hipcc flags]    UNIT: gic_bcx | gic_bc7 | gic_bc7enc | gic_bc6h
#   VAR_REV=<git rev>: build the unit's source as of that revision (an A/B baseline)
#   VAR_SRC=<file>: build that file in place of the unit's source
set -e
NAME=$1; UNIT=$2; shift 2
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
cd $D
T=$(mktemp -d)
SRC=csrc/$UNIT.hip
if [ -n "$VAR_REV" ]; then SRC=csrc/_var_$UNIT.hip; git show $VAR_REV:gfx_imagecompress_amd/csrc/$UNIT.hip > $SRC; fi
if [ -n "$VAR_SRC" ]; then SRC=csrc/_var_$UNIT.hip; cp "$VAR_SRC" $SRC; fi
/opt/rocm/bin/hipcc $F "$@" -c $SRC -o $T/$UNIT.o
if [ -n "$VAR_REV$VAR_SRC" ]; then rm -f $SRC; fi
OBJS=""
for u in gic_bcx gic_bc7 gic_bc7enc gic_bc6h gic_api gic_multi gic_pipeline; do
  if [ $u = $UNIT ]; then OBJS="$OBJS $T/$u.o"; else OBJS="$OBJS build/$u.o"; fi
done
mkdir -p ../gpurun_var/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_var/$NAME/lib.so $OBJS -L/opt/rocm/lib -lrccl -lpthread
rm -rf $T
echo built $NAME
