# Build a variant of the library with another gic_bcx.hip into gpurun_var/<name>/lib.so
# (travels to the box; git-ignored).   tools/build_bcx_variant.sh NAME BCX_SRC [extra hipcc flags]
set -e
NAME=$1; SRC=$(realpath $2); shift 2
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
cd $D
cp $SRC csrc/_v_bcx.hip
/opt/rocm/bin/hipcc $F "$@" -c csrc/_v_bcx.hip -o /tmp/_v_bcx.o
rm -f csrc/_v_bcx.hip
mkdir -p ../gpurun_var/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_var/$NAME/lib.so /tmp/_v_bcx.o build/gic_bc7.o build/gic_bc7enc.o build/gic_bc6h.o build/gic_api.o build/gic_multi.o -L/opt/rocm/lib -lrccl -lpthread
echo built $NAME
