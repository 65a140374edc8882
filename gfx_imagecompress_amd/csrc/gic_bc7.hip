// gic_bc7.hip -- placeholder (BC7 pipeline lands in the next commit)
#include "gic_common.h"
namespace gic {
hipError_t launch_bc7_image(const Geometry &, const gic_options &, void *, double *, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_bc7_blocks(const float *, uint32_t, const gic_options &, void *, double *, hipStream_t) { return hipErrorNotSupported; }
}
