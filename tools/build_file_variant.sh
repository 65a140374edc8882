# Build a variant of the library with one source file replaced (or rebuilt with
# extra flags) into gpurun_dbg/<name>/lib.so.
#   tools/build_file_variant.sh NAME UNIT SRC [extra hipcc flags]
# UNIT: gic_bcx | gic_bc7 | gic_bc7enc | gic_bc6h (the object it replaces)
set -e
NAME=$1; UNIT=$2; SRC=$3; shift 3
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math"
cd $D
cp $SRC csrc/_fv_$UNIT.hip
/opt/rocm/bin/hipcc $F "$@" -c csrc/_fv_$UNIT.hip -o /tmp/_fv_$NAME.o
rm -f csrc/_fv_$UNIT.hip
OBJS=""
for u in gic_bcx gic_bc7 gic_bc7enc gic_bc6h gic_api; do
  if [ $u = $UNIT ]; then OBJS="$OBJS /tmp/_fv_$NAME.o"; else OBJS="$OBJS build/$u.o"; fi
done
mkdir -p ../gpurun_dbg/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_dbg/$NAME/lib.so $OBJS
echo built $NAME
