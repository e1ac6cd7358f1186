#include "hgp_pass_dispatch.hpp"
namespace hgp {
template hipError_t launch_pass<float>(int, int, int, const PassDesc&, int64_t, hipStream_t);
template PassGeom pass_geom<float>(int, int);
template hipError_t launch_rowt<float>(int, int, int, const PassDesc&, hipStream_t, int);
template int rowt_pairs<float>(int, int);
template int rowt_threads<float>(int, int);
template int rowt_fits<float>(int, int);
template int rowt_group<float>(int);
template int linet_fits<float>(int);
template hipError_t launch_linet<float>(int, int, const PassDesc&, hipStream_t);
}
