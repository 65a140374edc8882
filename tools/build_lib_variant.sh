# Build the whole library with extra hipcc flags into gpurun_var/<name>/lib.so
# (travels to the box; git-ignored).   tools/build_lib_variant.sh NAME [extra hipcc flags]
set -e
NAME=$1; shift
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
cd $D
T=$(mktemp -d)
for f in gic_bcx gic_bc7 gic_bc7enc gic_bc6h; do /opt/rocm/bin/hipcc $F "$@" -c csrc/$f.hip -o $T/$f.o & done
wait
mkdir -p ../gpurun_var/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_var/$NAME/lib.so $T/gic_bcx.o $T/gic_bc7.o $T/gic_bc7enc.o $T/gic_bc6h.o build/gic_api.o build/gic_multi.o -L/opt/rocm/lib -lrccl -lpthread
rm -rf $T
echo built $NAME
