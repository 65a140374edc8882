# Build a variant of the BC7 library into gpurun_var/<name>/lib.so (travels to the box; git-ignored).
#   tools/build_variant.sh NAME WAVE_INC HIP_SRC [extra hipcc flags]
# WAVE_INC / HIP_SRC: paths of the bc7_wave.inc / gic_bc7.hip to use; QUANT_INC=path overrides bc7_quant.inc.
set -e
NAME=$1; WAVE=$2; HIP=$3; shift 3
D=/root/repo/gfx_imagecompress_amd
F="-I../include -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-fast-math -fno-slp-vectorize"
cd $D
cp $WAVE csrc/_v_wave.inc
cp ${QUANT_INC:-csrc/bc7_quant.inc} csrc/_v_quant.inc
sed 's/#include "bc7_wave.inc"/#include "_v_wave.inc"/; s/#include "bc7_quant.inc"/#include "_v_quant.inc"/' $HIP > csrc/_v.hip
/opt/rocm/bin/hipcc $F "$@" -c csrc/_v.hip -o /tmp/_v_bc7.o
mkdir -p ../gpurun_var/$NAME
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../gpurun_var/$NAME/lib.so build/gic_bcx.o /tmp/_v_bc7.o build/gic_bc7enc.o build/gic_bc6h.o build/gic_api.o build/gic_multi.o -L/opt/rocm/lib -lrccl -lpthread
rm -f csrc/_v.hip csrc/_v_wave.inc csrc/_v_quant.inc
echo built $NAME
