#include "hgp_pass_dispatch.hpp"
namespace hgp {
template hipError_t launch_pass<double>(int, int, int, const PassDesc&, int64_t, hipStream_t);
template PassGeom pass_geom<double>(int, int);
template hipError_t launch_rowt<double>(int, int, int, const PassDesc&, hipStream_t, int);
template int rowt_pairs<double>(int, int);
template int rowt_threads<double>(int, int);
template int rowt_fits<double>(int, int);
template int rowt_group<double>(int);
template int linet_fits<double>(int);
template hipError_t launch_linet<double>(int, int, const PassDesc&, hipStream_t);
}
