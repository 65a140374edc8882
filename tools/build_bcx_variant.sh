# Build a variant of the library with another gic_bcx.hip into gpurun_dbg/<name>/lib.so.
#   tools/build_bcx_variant.sh NAME BCX_SRC [extra hipcc flags]
set -e
NAME=$1; SRC=$2; shift 2
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math"
cd $D
cp $SRC csrc/_vb.hip
/opt/rocm/bin/hipcc $F "$@" -c csrc/_vb.hip -o /tmp/_vb_$NAME.o
rm -f csrc/_vb.hip
mkdir -p ../gpurun_dbg/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_dbg/$NAME/lib.so /tmp/_vb_$NAME.o build/gic_bc7.o build/gic_bc7enc.o build/gic_bc6h.o build/gic_api.o
echo built $NAME
