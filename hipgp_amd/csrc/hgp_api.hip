// hgp_api.hip — plan object and the extern "C" ABI of libhipgp.so (see include/hipgp.h).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/hipgp.h"
#include "hgp_internal.hpp"

using namespace hgp;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t _e = (expr);                                                                        \
    if (_e != hipSuccess)                                                                          \
      return fail(HGP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));                   \
  } while (0)

#define HGP_TRY(expr)                                                                              \
  do {                                                                                             \
    int _rc = (expr);                                                                              \
    if (_rc != 0) return _rc;                                                                      \
  } while (0)

// smallest 3 * 2^k >= v with k >= 3 (a transform half-length 3 * 2^(k-1) >= 12, hgp_fft.hpp is_tri)
int64_t next_tri(int64_t v) {
  int64_t t = 24;
  while (t < v) t <<= 1;
  return t;
}

int64_t next_pow2(int64_t v) {
  int64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  int ensure(size_t need) {
    if (need <= bytes) return 0;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&ptr, need);
    if (e != hipSuccess) return fail(HGP_E_OOM, std::string("hipMalloc(") + std::to_string(need) + "): " + hipGetErrorString(e));
    bytes = need;
    return 0;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
  }
};

// hgp_rowdot's partial-sum scratch (one per host thread and device, never freed: a few KB-MB)
struct RowdotScratch {
  int device = -1;
  DevBuf buf;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
  bool used = false;
  RowdotScratch() = default;
  RowdotScratch(RowdotScratch&& o) noexcept : device(o.device), ev(o.ev), last(o.last), used(o.used) {
    buf.ptr = o.buf.ptr; buf.bytes = o.buf.bytes; o.buf.ptr = nullptr; o.buf.bytes = 0; o.ev = nullptr;
  }
};

}  // namespace

struct hgp_plan {
  int device = 0;
  int dtype = HGP_F32;
  hipStream_t stream = nullptr;
  int d = 0;                              // effective dims (axes with m > 1)
  int ndim_user = 0;
  int64_t m[3] = {1, 1, 1}, n[3] = {1, 1, 1}, LK[3] = {1, 1, 1}, LR[3] = {1, 1, 1};
  int64_t M = 1, Mp = 1, prodLK = 1, prodLR = 1;
  size_t esz = 4;
  // tables
  DevBuf twK[3], twR[3], tw64K[3], tw64R[3];
  // fp64 twiddles of the radix-2 levels of fft_lines_f64 for lines longer than one CU's LDS:
  // level j >= 1 of axis a holds W_{L/2^j} (L = L_K: tw64Kl, L_R: tw64Rl), down to the base pass
  static constexpr int NLEV = 8;
  DevBuf tw64Kl[3][NLEV], tw64Rl[3][NLEV];
  DevBuf bsPre[3], bsPost[3], bsFilt[3];   // Bluestein DCT-I tables per axis (fp64)
  // spectra
  DevBuf specK, specI, specR, Dm3;
  bool have_spec = false;
  // R / R^T spectrum real (the filter embedded evenly: L_R >= 2n - 1 on every axis, d >= 2):
  // real-spectrum conv passes instead of complex ones, half the spectrum bytes
  bool r_real = false;
  // fp64 plans whose L_R lines exceed one CU's LDS (L_R / 2 > 8192): R / R^T on the full fp64
  // grid (run_op_grid: fwd_grid_f64's radix-2 step), spectrum in the transforms' stored order
  bool grid_r = false;
  // plans with an axis longer than the passes hold (> 8192 points, both dtypes): K / C^-1 on the
  // full fp64 L_K grid as well (run_op_grid), spectrum in the transforms' stored order: K in the
  // real parts, C^-1 in the imaginary parts of specKg
  bool grid_k = false;
  DevBuf specRg, specKg, gridA, gridB;
  double clamp_min = 1e-6;                // of the last set_column (the clamp's gradient mask)
  DevBuf nclamp;
  // scratch
  DevBuf ws1, ws2, set1, set2, setM1, setM2, setC;
  // CG state
  DevBuf r, z, p, Ap, part_op, part_u, part_f, scal, flags, bT, xT;
  // slab-sharded PCG (hgp_slab_cg_*): fused-dot / update partials and per-RHS alpha / beta
  DevBuf slab_part, slab_coef;
  int64_t cg_nrhs = 0;
  int cg_precond = 0, cg_layout = 0;
  void* cg_x_user = nullptr;
  void* cg_x = nullptr;
  bool cg_active = false;
  int cg_rs_par = 0;                      // which of the two rs buffers the next step reads
  int cg_step = 0;                        // steps queued since hgp_pcg_begin
  // 2-D RHS-chunk budget: 2 GiB measured best at C4 (PCG(20) 213 -> 205 ms vs 1 GiB; C3 and the C4
  // single ops flat; profiles/r5_i_ws_budget.txt)
  int64_t ws_budget = (int64_t)2 << 30;
  int64_t ws3_budget = (int64_t)4 << 30;  // 3-D default (hgp_plan_create: from the device's memory)
  bool ws_explicit = false;               // HGP_WS_MB given: the byte budget alone sets the chunks
  // 2-D operators run their RHS chunks on `nstreams` streams (the plan's own + side streams),
  // so one chunk's compute-heavy column pass overlaps another's memory-heavy row passes
  int nstreams = 2;
  // the 2-D preconditioned PCG chains K p and C^-1 r per RHS chunk (pcg_step_t; HGP_CHAIN_PCG=1).
  // Off by default: measured slower at every 2-D config (PCG(20) C2 14.9 -> 15.2 ms, C3 390 ->
  // 395 ms, C4 215.4 -> 218 ms; profiles/r5_e_kn_phases_chain.txt)
  bool chain_pcg = false;
  // pack the 2-D K / C^-1 intermediate's real DC and Nyquist columns into one (PassDesc::dcny;
  // HGP_DCNY=0: off)
  bool dcny_pack = true;
  // the fp32 1024-point K / C^-1 column conv with two lines per wave, radix-32 stages (LAY_CONTIG2,
  // HGP_CONV_P32=1): one LDS exchange per transform instead of two, but 2 waves per SIMD instead of 4
  // (the LDS images bound a CU to 16 lines either way) -- measured slower, C2 column pass 0.149 ->
  // 0.171 ms (profiles/r6r_conv_p32_ab.txt); kept as an opt-in for that measurement
  bool conv_p32 = false;
  // HGP_BALANCED_CHUNKS=1: RHS chunks of equal size, their count a multiple of the stream count
  // (run_op), so the streams carry equal work.  Off: measured neutral with the settings
  // interleaved on one box (C3 PCG(20) 391 vs 390 ms, C4 209 vs 209 ms, C3 / C4 K op +-0.3 %;
  // profiles/r6i_balanced_chunks_ab_interleaved.jsonl) -- the fixed Qc-sized chunks stay
  bool balanced_chunks = false;
  hipStream_t side[3] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_fork = nullptr, ev_join[3] = {nullptr, nullptr, nullptr};
  // hipGraph of a repeated hgp_toeplitz_apply (same op, buffers, RHS count, workspaces, stream):
  // the second identical call is captured, later ones replay it (no per-kernel launch gaps)
  struct ApplyKey {
    int op = -1;
    const void* x = nullptr;
    void* y = nullptr;
    int64_t nrhs = 0;
    hipStream_t stream = nullptr;
    // every plan-owned buffer an op's launches address (workspaces, the full-grid route's
    // buffers, the spectra): a reallocation of any of them -- e.g. R^T on a grid_k plan growing
    // gridA / gridB past K's size -- must invalidate a captured graph
    static constexpr int NB = 9;
    const void* buf[NB] = {};
    bool operator==(const ApplyKey& o) const {
      if (!(op == o.op && x == o.x && y == o.y && nrhs == o.nrhs && stream == o.stream)) return false;
      for (int i = 0; i < NB; ++i)
        if (buf[i] != o.buf[i]) return false;
      return true;
    }
  };
  void key_buffers(ApplyKey& k) const {
    const DevBuf* b[ApplyKey::NB] = {&ws1, &ws2, &gridA, &gridB, &specK, &specI, &specR, &specRg, &specKg};
    for (int i = 0; i < ApplyKey::NB; ++i) k.buf[i] = b[i]->ptr;
  }
  ApplyKey last_apply, graph_key;
  hipGraphExec_t graph_exec = nullptr;
  hipStream_t cap_stream = nullptr;       // captures run here (torch's default stream cannot capture)
  bool use_graphs = true;
  void drop_graph() {
    if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
    graph_exec = nullptr;
    graph_key = ApplyKey();
  }

  ~hgp_plan() {
    drop_graph();
    if (cap_stream) (void)hipStreamDestroy(cap_stream);
    for (int a = 0; a < 3; ++a) {
      twK[a].release(); twR[a].release(); tw64K[a].release(); tw64R[a].release();
      for (int j = 0; j < NLEV; ++j) { tw64Kl[a][j].release(); tw64Rl[a][j].release(); }
      bsPre[a].release(); bsPost[a].release(); bsFilt[a].release();
    }
    DevBuf* bufs[] = {&specK, &specI, &specR, &specRg, &specKg, &gridA, &gridB, &Dm3, &nclamp, &ws1, &ws2, &set1, &set2, &setM1, &setM2, &setC,
                      &r, &z, &p, &Ap, &part_op, &part_u, &part_f, &scal, &flags, &bT, &xT};
    for (DevBuf* b : bufs) b->release();
    for (int i = 0; i < 3; ++i) {
      if (side[i]) (void)hipStreamDestroy(side[i]);
      if (ev_join[i]) (void)hipEventDestroy(ev_join[i]);
    }
    if (ev_fork) (void)hipEventDestroy(ev_fork);
  }
};

namespace {

// 3-D operators' default workspace budget: an eighth of the device's memory, at most 32 GiB (36 GB
// of a 288 GB MI355X).  The R / R^T intermediates of a C5 grid are 1 GB per RHS; with this budget
// each of the two streams takes its whole half of the 25 RHS in one chunk, so the axis-0 pass
// fetches the complex spectrum (0.9 GB) twice per op instead of 13 times, and each pass launches
// twice instead of 13 times: C5 R^T 20.8 -> 19.6 ms (4 GiB -> 26 GB, profiles/r3_m_rt_ws.txt).
#ifndef HGP_WS3_MAX
#define HGP_WS3_MAX ((int64_t)32 << 30)
#endif

// op geometry: per-axis input/output lengths and transform length
struct OpGeom {
  int64_t in[3], out[3], L[3];
  int64_t in_M, out_M;
  const DevBuf* tw;        // per-axis twiddle tables (plan dtype)
  const void* spec;
  int spec_kind;
};

OpGeom op_geom(const hgp_plan* P, int op) {
  OpGeom g;
  for (int a = 0; a < 3; ++a) { g.in[a] = 1; g.out[a] = 1; g.L[a] = 1; }
  g.in_M = g.out_M = 1;
  for (int a = 0; a < P->d; ++a) {
    const bool rtype = (op == HGP_OP_RT || op == HGP_OP_R);
    g.L[a] = rtype ? P->LR[a] : P->LK[a];
    g.in[a] = (op == HGP_OP_R) ? P->n[a] : P->m[a];
    g.out[a] = (op == HGP_OP_RT) ? P->n[a] : P->m[a];
    g.in_M *= g.in[a];
    g.out_M *= g.out[a];
  }
  g.tw = (op == HGP_OP_RT || op == HGP_OP_R) ? P->twR : P->twK;
  if (op == HGP_OP_K) { g.spec = P->specK.ptr; g.spec_kind = SPEC_REAL; }
  else if (op == HGP_OP_CINV) { g.spec = P->specI.ptr; g.spec_kind = SPEC_REAL; }
  else if (op == HGP_OP_RT) { g.spec = P->specR.ptr; g.spec_kind = P->r_real ? SPEC_REAL : SPEC_CPLX; }
  else { g.spec = P->specR.ptr; g.spec_kind = P->r_real ? SPEC_REAL : SPEC_CPLX_CONJ; }
  return g;
}

template <typename T>
int launch(int H, int mode, int lay, const PassDesc& d, int64_t lines_contig, hipStream_t s) {
  const PassGeom g = pass_geom<T>(H, lay);
  if (g.C == 0) return fail(HGP_E_UNSUPPORTED, "transform half-length " + std::to_string(H) + " not supported");
  // forward transforms and complex-spectrum conv passes fold an input longer than H (hgp_pass.hpp CAN_FOLD)
  const bool can_fold = mode == PASS_FWD || mode == PASS_CONVC;
  if (mode != PASS_INV && (can_fold ? d.in.len > 2 * H : d.in.len > H))
    return fail(HGP_E_ARG, "internal: pass input length " + std::to_string(d.in.len) + " > H = " + std::to_string(H));
  int64_t nb;
  if (lay == LAY_STRIDED || lay == LAY_SEG_S) nb = (int64_t)d.Q * d.Rn * ((d.In + g.C - 1) / g.C);
  else nb = (lines_contig + g.C - 1) / g.C;
  if (nb <= 0) return 0;
  if (nb > 0x7fffffff) return fail(HGP_E_UNSUPPORTED, "grid too large");
  hipError_t e = launch_pass<T>(H, mode, lay, d, nb, s);
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("k_pass launch: ") + hipGetErrorString(e));
  return 0;
}

PassDesc base_desc() {
  PassDesc d;
  std::memset(&d, 0, sizeof(d));
  return d;
}

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// compact half-spectrum row length of the last (real) axis: >= H+1, 64-byte aligned rows
int64_t compact_stride(int64_t L) { return round_up(L / 2 + 1, 8); }

// Side streams + fork/join events of a plan (created on first use, on the plan's device).
int ensure_side_streams(hgp_plan* P, int n) {
  for (int i = 0; i < n - 1 && i < 3; ++i) {
    if (P->side[i] == nullptr) HIP_TRY(hipStreamCreateWithFlags(&P->side[i], hipStreamNonBlocking));
    if (P->ev_join[i] == nullptr) HIP_TRY(hipEventCreateWithFlags(&P->ev_join[i], hipEventDisableTiming));
  }
  if (P->ev_fork == nullptr) HIP_TRY(hipEventCreateWithFlags(&P->ev_fork, hipEventDisableTiming));
  return 0;
}

// Fused PCG epilogue of the 2-D row-inverse pass (hgp_rows.hpp EPI_XR / EPI_P): the operator
// output y updates the CG vectors (x, r, p: row layout, nrhs x M) instead of being stored.
struct RowEpi {
  int mode;
  void* r;
  void* x;
  void* p;
  const void* coef;   // per-RHS alpha (EPI_XR, EPI_R) or beta (EPI_XP), when sp == nullptr
  void* part;         // EPI_XR / EPI_R: r.r partials [q][row block]
  // in-kernel alpha / beta (PassDesc::cg_sp): spectral partials [q][np], rs in / out per RHS
  const void* sp = nullptr;
  int np = 0;
  const void* rs = nullptr;
  void* rs_out = nullptr;
  const void* coef2 = nullptr;   // EPI_XP: alpha per RHS
  void* alpha_out = nullptr;     // EPI_R (in-kernel alpha): where EPI_XP reads it
  int fix = 0;                   // EPI_XP: PassDesc::cg_fix
};

// the chunk (first RHS q0) view of an epilogue's in-kernel CG scalar
template <typename T>
void set_cg_scalar(PassDesc& D, const RowEpi* epi, int64_t q0) {
  D.cg_coef2 = epi->coef2 ? reinterpret_cast<const T*>(epi->coef2) + q0 : nullptr;
  D.cg_alpha_out = epi->alpha_out ? reinterpret_cast<T*>(epi->alpha_out) + q0 : nullptr;
  D.cg_fix = epi->fix;
  if (epi->sp == nullptr) return;
  D.cg_sp = reinterpret_cast<const T*>(epi->sp) + q0 * epi->np;
  D.cg_np = epi->np;
  D.cg_rs = reinterpret_cast<const T*>(epi->rs) + q0;
  D.cg_rs_out = epi->rs_out ? reinterpret_cast<T*>(epi->rs_out) + q0 : nullptr;
}

// Called between the 2-D column pass and the row-inverse pass of each RHS chunk (q0, qn):
// computes the chunk's alpha / beta from the column pass's spectral dots.
using MidFn = std::function<void(int64_t, int, hipStream_t)>;

// A second operator chained onto a 2-D K op per RHS chunk (the fused PCG iteration, pcg_step_t):
// K's row-inverse pass runs EPI_RF (r update + the forward row transform of the new r into the
// chunk's intermediate), then this op's axis-0 pass (spectrum `spec`, spectral dots into
// `spart`), `mid`, and its row-inverse pass with epilogue `epi` -- K p and C^-1 r of one
// iteration back to back on each chunk's stream, r never re-read from HBM.
struct PairOp {
  const void* spec;
  void* spart;
  const RowEpi* epi;
  const MidFn* mid;
};

// y = op(x) on RHS [0, nrhs); optional fused dot with `dotv` into partial[b][rn_last].
// Every RHS is processed on its own (no two RHS share an FFT).  only_pass >= 0 runs a single
// pass of the sequence (profiling).  2-D only: `spart` receives the column pass's spectral
// dots <x, op x> per (RHS, compact column) [q][L_1/2 + 1]; `epi` replaces the output store by
// the fused PCG update, `mid` runs between the column pass and the row-inverse pass.
int fwd_grid_f64(hgp_plan* P, const int64_t* L, const DevBuf* tw64, double2* a, double2* b, double2** result,
                 const int* done = nullptr);

// The full-grid route, one RHS at a time on the full fp64 L-grid of the operator:
// y = crop(IFFT(S' FFT(pad x))), the inverse as conj(FFT(conj Y)) / N (the 1/N is in the stored
// spectrum).  R / R^T of grid_r plans on the L_R grid (S' = S for R^T, conj(S) for R, specRg);
// K / C^-1 of grid_k plans on the L_K grid (S' = Re / Im of specKg, the packed K + i C^-1
// transform).  Exact like the pass route (same spectra, fp64 throughout); memory 2 prod(L)
// complex fp64.  A fused dot (dotv) becomes per-RHS row-chunk partials of y . dotv
// (rowdot_part: update_np(out M) per RHS, the unfused PCG's op_np).
template <typename T>
int run_op_grid(hgp_plan* P, int op, const void* x, void* y, int64_t nrhs, const void* dotv, void* partial,
                const int* done) {
  hipStream_t s = P->stream;
  const int d = P->d;
  const bool rtype = op == HGP_OP_R || op == HGP_OP_RT;
  const int64_t* Lg = rtype ? P->LR : P->LK;
  const DevBuf* tw64 = rtype ? P->tw64R : P->tw64K;
  const int64_t N = rtype ? P->prodLR : P->prodLK;
  HGP_TRY(P->gridA.ensure((size_t)N * sizeof(double2)));
  HGP_TRY(P->gridB.ensure((size_t)N * sizeof(double2)));
  double2* A = reinterpret_cast<double2*>(P->gridA.ptr);
  double2* B = reinterpret_cast<double2*>(P->gridB.ptr);
  GridDims gi, go;
  gi.d = go.d = d;
  int64_t inM = 1, outM = 1;
  for (int a = 0; a < 3; ++a) {
    gi.L[a] = go.L[a] = Lg[a];
    gi.n[a] = go.n[a] = P->n[a];
    gi.m[a] = (op == HGP_OP_R) ? P->n[a] : P->m[a];
    go.m[a] = (op == HGP_OP_RT) ? P->n[a] : P->m[a];
    if (a < d) { inM *= gi.m[a]; outM *= go.m[a]; }
  }
  const double2* S = reinterpret_cast<const double2*>(rtype ? P->specRg.ptr : P->specKg.ptr);
  const int mode = op == HGP_OP_R ? 1 : op == HGP_OP_RT ? 0 : op == HGP_OP_K ? 2 : 3;
  const size_t es = P->esz;
  for (int64_t q = 0; q < nrhs; ++q) {
    grid_embed(P->dtype, static_cast<const char*>(x) + (size_t)(q * inM) * es, gi, N, A, s, done);
    double2* F = nullptr;
    HGP_TRY(fwd_grid_f64(P, Lg, tw64, A, B, &F, done));
    double2* other = (F == A) ? B : A;
    grid_mul_unperm(F, S, gi, N, mode, other, s, done);
    double2* Z = nullptr;
    HGP_TRY(fwd_grid_f64(P, Lg, tw64, other, F, &Z, done));
    grid_crop(P->dtype, Z, go, outM, static_cast<char*>(y) + (size_t)(q * outM) * es, s, done);
  }
  if (dotv != nullptr && partial != nullptr)
    rowdot_part<T>(y, dotv, partial, nrhs, outM, update_np(outM), s);
  HIP_TRY(hipGetLastError());
  return 0;
}

bool grid_route(const hgp_plan* P, int op) {
  return (op == HGP_OP_R || op == HGP_OP_RT) ? P->grid_r : P->grid_k;
}

template <typename T>
int run_op(hgp_plan* P, int op, const void* x, void* y, int64_t nrhs, const void* dotv, void* partial,
           const int* done, int only_pass = -1, void* spart = nullptr, const RowEpi* epi = nullptr,
           const MidFn* mid = nullptr, const PairOp* pair = nullptr) {
  if (grid_route(P, op)) {
    if (spart != nullptr || epi != nullptr || mid != nullptr || only_pass >= 0)
      return fail(HGP_E_UNSUPPORTED, "internal: the full-grid route has no fused PCG epilogue or pass split");
    // after the break (`done` set) every transform / embed / crop kernel of the route is a device
    // no-op, so the iterations up to maxiter cost launches only; the dot partials it may still
    // write are never read
    return run_op_grid<T>(P, op, x, y, nrhs, dotv, partial, done);
  }
  const OpGeom g = op_geom(P, op);
  const int d = P->d;
  const int conv_mode = g.spec_kind == SPEC_REAL ? PASS_CONV : PASS_CONVC;
  const size_t cs = sizeof(C2<T>);
  const int64_t Sl = compact_stride(g.L[d - 1]);
  // per-RHS workspace (complex elements)
  int64_t B1 = 0, B2 = 0;
  // 2-D: column-major intermediate W[q][c][i0], c < H1 + 1, column pitch S0 (hgp_rows.hpp);
  // rows whose row-pair kernels do not fit one CU's LDS (fp64 H >= 8192) take the generic
  // sequence instead: row pairs -> row-major [q][i0][c] -> strided axis-0 conv -> row pairs
  const bool gen2 = d == 2 && !rowt_fits<T>((int)(g.L[1] / 2), 1);
  // long fp32 rows: the 2-D intermediate in the grouped-column layout (hgp_rows.hpp)
  const int G2 = (d == 2 && !gen2) ? rowt_group<T>((int)(g.L[1] / 2)) : 1;
  const int64_t S0 = (d >= 2) ? round_up(std::max(g.in[0], g.out[0]), 16) : 0;   // axis-0 pitch
  if (d == 2) B1 = gen2 ? std::max(g.in[0], g.out[0]) * Sl : (g.L[1] / 2 + G2) / G2 * G2 * S0;
  if (gen2 && (spart != nullptr || epi != nullptr || mid != nullptr))
    return fail(HGP_E_ARG, "internal: the generic 2-D sequence has no fused PCG epilogue");
  if (pair != nullptr && (d != 2 || gen2 || epi == nullptr || epi->mode != EPI_R || only_pass >= 0))
    return fail(HGP_E_ARG, "internal: a chained operator needs the 2-D row-pair sequence and an EPI_R epilogue");
  // 3-D (hgp_lines.hpp): the (i1, i2) plane of every (RHS, i0) goes through the 2-D row-pair
  // kernels -> W1 [q][i0][c2][i1] (column pitch S1); transposing axis-1 line passes <->
  // W2 [q][c2][k1][i0] (axis-0 pitch S0), whose axis-0 lines the contiguous conv pass takes.
  // Kernels that do not fit one CU's LDS (fp64 at H >= 8192) take the row-major 5-pass
  // sequence with strided middle passes instead (gen3).
  const bool gen3 = d == 3 && (!rowt_fits<T>((int)(g.L[2] / 2), 0) || !linet_fits<T>((int)(g.L[1] / 2)));
  const int64_t S1 = (d == 3) ? round_up(std::max(g.in[1], g.out[1]), 16) : 0;
  if (d == 3) {
    const int64_t P0 = std::max(g.in[0], g.out[0]), NC2 = g.L[2] / 2 + 1;
    B1 = gen3 ? std::max(g.in[0] * g.in[1], g.out[0] * g.out[1]) * Sl : P0 * NC2 * S1;
    B2 = gen3 ? P0 * g.L[1] * Sl : NC2 * g.L[1] * S0;
    // the axis-0 / middle passes address one RHS's W2 with 32-bit element offsets
    if (B2 >= ((int64_t)1 << 31)) return fail(HGP_E_UNSUPPORTED, "3-D grid too large: one right-hand side's intermediate exceeds 2^31 values");
  }
  if (gen3 && (spart != nullptr || epi != nullptr || mid != nullptr))
    return fail(HGP_E_ARG, "internal: the generic 3-D sequence has no fused PCG epilogue");
  // the 2-D row passes address one RHS's intermediate slab (and the contiguous pass one line)
  // with 32-bit byte offsets from a scalar base (raw buffer accesses, hgp_rows.hpp)
  if (d == 2 && !gen2 && B1 * (int64_t)cs >= ((int64_t)1 << 31))
    return fail(HGP_E_UNSUPPORTED, "2-D grid too large: one right-hand side's intermediate exceeds 2 GiB");
  // RHS chunks: 2-D ops spread them over NS streams, chunk j on stream (and workspace slot)
  // j % NS; each chunk's RHS are processed entirely on its stream (no cross-stream data).
  const int NS = (d >= 2 && only_pass < 0) ? (int)std::min<int64_t>(std::max(1, P->nstreams), nrhs) : 1;
  int64_t Qc = nrhs;
  if (B1 + B2 > 0) {
    const int64_t per = (B1 + B2) * (int64_t)cs;
    // 3-D: a larger default budget, so the axis-0 pass's spectrum lines (C5 R^T: 0.9 GB) are
    // fetched once per chunk of several RHS instead of once per RHS
    const int64_t budget = (d == 3 && !P->ws_explicit) ? std::max<int64_t>(P->ws_budget, P->ws3_budget) : P->ws_budget;
    Qc = std::max<int64_t>(1, std::min<int64_t>((nrhs + NS - 1) / NS, budget / (per * NS)));
    // Infinity-Cache-resident chunks: where 8 RHS of a 2-D intermediate fit in ~72 MiB, each
    // stream works on 8 RHS at a time, so the intermediate a column pass writes is still in the
    // 256 MiB Infinity Cache when the row-inverse pass reads it (C2: row inverse 4.2 -> 5.0 TB/s,
    // K matvec +4-6 %, tools/gpu_env_ab.sh).  Larger grids keep the byte budget (fewer RHS per
    // chunk there cost more in launch tails than the cache gains: C3 / C4 measured slower).
    if (d == 2 && !P->ws_explicit && per * 8 <= ((int64_t)72 << 20)) Qc = std::min<int64_t>(Qc, 8);
    HGP_TRY(P->ws1.ensure((size_t)(B1 * Qc * NS) * cs));
    if (B2) HGP_TRY(P->ws2.ensure((size_t)(B2 * Qc * NS) * cs));
  }
  hipStream_t streams[4] = {P->stream, nullptr, nullptr, nullptr};
  if (NS > 1) {
    HGP_TRY(ensure_side_streams(P, NS));
    HIP_TRY(hipEventRecord(P->ev_fork, P->stream));
    for (int i = 1; i < NS; ++i) {
      streams[i] = P->side[i - 1];
      HIP_TRY(hipStreamWaitEvent(streams[i], P->ev_fork, 0));
    }
  }
  const T* xin = reinterpret_cast<const T*>(x);
  T* yout = reinterpret_cast<T*>(y);
  const T* dv = reinterpret_cast<const T*>(dotv);
  T* part = reinterpret_cast<T*>(partial);
  // fused-dot partials per RHS: one per output row pair (3-D: per pair of each i0 plane)
  const int64_t rows_out = (d == 1) ? 1 : (d == 2 ? g.out[0] : g.out[0] * g.out[1]);
  const int64_t rn_last = (d == 1) ? 1 : (d == 3 && !gen3) ? g.out[0] * ((g.out[1] + 1) / 2) : (rows_out + 1) / 2;

  // chunk j of nch: RHS [j nrhs / nch, (j + 1) nrhs / nch).  Balanced (HGP_BALANCED_CHUNKS=1): nch = ceil(nrhs /
  // Qc) rounded up to a multiple of NS and sizes that differ by at most one, so the NS streams get
  // equal work (fixed Qc-sized chunks left e.g. C3's 200 RHS as 63 + 63 + 63 + 11: 126 RHS on one
  // stream, 74 on the other; C4's 25 as 8 + 8 + 8 + 1).  Every chunk still fits its Qc workspace slot.
  int64_t nch = (nrhs + Qc - 1) / Qc;
  if (P->balanced_chunks && NS > 1 && nch > 1) nch = (nch + NS - 1) / NS * NS;
  auto chunk_q0 = [&](int64_t j) -> int64_t {
    return P->balanced_chunks ? j * nrhs / nch : std::min(nrhs, j * Qc);
  };
  for (int64_t chunk = 0; chunk < nch; ++chunk) {
    const int64_t q0 = chunk_q0(chunk);
    const int qn = (int)(chunk_q0(chunk + 1) - q0);
    if (qn <= 0) continue;
    const int slot = (int)(chunk % NS);
    hipStream_t st = streams[slot];
    int pass_no = 0;
    auto run = [&](int H, int mode, int lay, PassDesc& D, int64_t lines) -> int {
      const int me = pass_no++;
      if (only_pass >= 0 && only_pass != me) return 0;
      return launch<T>(H, mode, lay, D, lines, st);
    };
    const T* xi = xin + q0 * g.in_M;
    T* yo = yout + q0 * g.out_M;
    const T* dvc = dv ? dv + q0 * g.out_M : nullptr;
    T* pc = part ? part + q0 * rn_last : nullptr;

    if (d == 1) {
      PassDesc D = base_desc();
      D.in = View{(void*)xi, g.in_M, 0, 1, (int)g.in[0]};
      D.out = View{yo, g.out_M, 0, 1, (int)g.out[0]};
      D.dot = dvc; D.partial = pc;
      D.spec = g.spec; D.spec_kind = g.spec_kind; D.spec_i = 0; D.spec_r = 0; D.spec_p = 1;
      D.tw = g.tw[0].ptr; D.Q = qn; D.Rn = 1; D.In = 1; D.done = done;
      HGP_TRY(run((int)(g.L[0] / 2), conv_mode, LAY_R1, D, qn));
    } else if (d == 2 && gen2) {
      C2<T>* w1 = reinterpret_cast<C2<T>*>(P->ws1.ptr) + (int64_t)slot * Qc * B1;
      const int64_t H1 = g.L[1] / 2;
      PassDesc A = base_desc();     // FWD axis 1: row pairs -> w1 [q][i0][c1] (pitch Sl)
      A.in = View{(void*)xi, g.in_M, g.in[1], 1, (int)g.in[1]};
      A.out = View{w1, B1, Sl, 1, 0};
      A.tw = g.tw[1].ptr; A.Q = qn; A.Rn = (int)((g.in[0] + 1) / 2); A.nrows = (int)g.in[0]; A.done = done;
      HGP_TRY(run((int)H1, PASS_FWD, LAY_RP, A, (int64_t)qn * A.Rn));
      PassDesc Bd = base_desc();    // CONV axis 0 (strided, in place): lines c1, spectrum [c1][k0]
      Bd.in = View{w1, B1, 0, Sl, (int)g.in[0]};
      Bd.out = View{w1, B1, 0, Sl, (int)g.out[0]};
      Bd.spec = g.spec; Bd.spec_kind = g.spec_kind; Bd.spec_i = g.L[0]; Bd.spec_r = 0; Bd.spec_p = 1;
      Bd.tw = g.tw[0].ptr; Bd.Q = qn; Bd.Rn = 1; Bd.In = (int)(H1 + 1); Bd.done = done;
      HGP_TRY(run((int)(g.L[0] / 2), conv_mode, LAY_STRIDED, Bd, 0));
      PassDesc Cd = base_desc();    // INV axis 1: rebuild row pairs, crop, fused dot
      Cd.in = View{w1, B1, Sl, 1, (int)g.L[1]};
      Cd.out = View{yo, g.out_M, g.out[1], 1, (int)g.out[1]};
      Cd.dot = dvc; Cd.partial = pc;
      Cd.tw = g.tw[1].ptr; Cd.Q = qn; Cd.Rn = (int)((g.out[0] + 1) / 2); Cd.nrows = (int)g.out[0]; Cd.done = done;
      HGP_TRY(run((int)H1, PASS_INV, LAY_RP, Cd, (int64_t)qn * Cd.Rn));
    } else if (d == 2) {
      C2<T>* w1 = reinterpret_cast<C2<T>*>(P->ws1.ptr) + (int64_t)slot * Qc * B1;
      const int64_t H1 = g.L[1] / 2;
      auto run_rowt = [&](int inv, PassDesc& D, int epi_mode) -> int {
        const int me = pass_no++;
        if (only_pass >= 0 && only_pass != me) return 0;
        hipError_t e = launch_rowt<T>((int)H1, inv, epi_mode, D, st, 1);
        if (e == hipErrorNotSupported)
          return fail(HGP_E_UNSUPPORTED, "row transform of H = " + std::to_string(H1) +
                                             " points does not fit one CU's LDS in this dtype (use fp32)");
        if (e != hipSuccess) return fail(HGP_E_HIP, std::string("row pass launch: ") + hipGetErrorString(e));
        return 0;
      };
      // packed DC / Nyquist columns (PassDesc::dcny): K / C^-1 (real spectra) on the plain
      // layout, axis-0 lines of one wave, rows of >= 512 points (where the axis-0 pass's line
      // count per RHS decides its rounds of resident blocks; small grids keep every column)
      int dcny = 0;
      if (P->dcny_pack && G2 == 1 && (op == HGP_OP_K || op == HGP_OP_CINV) && H1 >= 256) {
        const PassGeom pg0 = pass_geom<T>((int)(g.L[0] / 2), LAY_CONTIG);
        if (pg0.C > 0 && pg0.threads / pg0.C <= 64) dcny = (int)(H1 / 2);
      }
      // A: FWD along axis 1, row pairs of each RHS -> column-major half spectra w1 [q][c1][i0]
      //    (grouped by G2 columns: w1 [q][c1 / G2][i0][c1 % G2])
      PassDesc A = base_desc();
      A.in = View{(void*)xi, g.in_M, g.in[1], 1, (int)g.in[1]};
      A.out = View{w1, B1, S0, 1, 0};
      A.tw = g.tw[1].ptr; A.Q = qn; A.Rn = (int)((g.in[0] + 1) / 2); A.nrows = (int)g.in[0]; A.done = done;
      A.dcny = dcny;
      HGP_TRY(run_rowt(0, A, EPI_OUT));
      // B: CONV along axis 0 = contiguous lines (q, c1), in place; spectrum [c1][k0]
      PassDesc Bd = base_desc();
      Bd.in = View{w1, B1, S0, 1, (int)g.in[0]};
      Bd.out = View{w1, B1, S0, 1, (int)g.out[0]};
      Bd.spec = g.spec; Bd.spec_kind = g.spec_kind; Bd.spec_i = 0; Bd.spec_p = 1; Bd.spec_r = g.L[0];
      Bd.tw = g.tw[0].ptr; Bd.Q = qn; Bd.Rn = (int)(H1 + 1); Bd.In = 1; Bd.done = done;
      Bd.dcny = dcny;
      if (spart != nullptr) {
        Bd.spart = reinterpret_cast<T*>(spart) + q0 * (H1 + 1);
        Bd.spart_mid = (int)(H1 / 2);
      }
      int b_lay = LAY_CONTIG;
      int64_t b_lines = 0;
      if (G2 > 1) {     // lines (column group, RHS, column in group): ceil(Rn / G2) G2 per RHS
        Bd.grp = G2;
        // G2 position-fast blocks per group (LAY_CONTIG_G).  HGP_GRP_BLOCKS=1: one block per
        // (group, RHS) with the columns interleaved over its threads (LAY_GRP*) -- coalesced
        // 512-B accesses, but measured slower (C4 CONV 2.97 -> 3.85 ms, C3 0.765 -> 0.82 ms:
        // 16-wave blocks / interleaved exchange images, profiles/r3_grouped_passtime.txt)
        // G2 = 4 is stored in the quad order (HGP_QUAD, hgp_rows.hpp wg_off<4>): LAY_CONTIG_Q, two
        // lines (one 64-B half of a group's units) per block
        const bool quad = HGP_QUAD && G2 == 4;
        const int glay = G2 == 2 ? LAY_GRP2 : (G2 == 4 && !quad) ? LAY_GRP4 : -1;
        static const bool grp_on = [] { const char* e = std::getenv("HGP_GRP_BLOCKS"); return e && std::atoi(e) == 1; }();
        const bool use_grp = glay >= 0 && grp_on && pass_geom<T>((int)(g.L[0] / 2), glay).C == G2;
        b_lay = use_grp ? glay : quad ? LAY_CONTIG_Q : LAY_CONTIG_G;
        b_lines = (int64_t)qn * ((H1 + G2) / G2) * G2;
      } else {
        // fp32 1024-point lines of exactly H rows in and out (no zero padding, no crop): two lines
        // per wave, radix-32 stages (LAY_CONTIG2); its wave-shared buffer resource needs the chunk's
        // intermediate below 2 GiB
        const bool two = std::is_same<T, float>::value && P->conv_p32 && conv_mode == PASS_CONV &&
                         g.L[0] == 2048 && g.in[0] == 1024 && g.out[0] == 1024 &&
                         (int64_t)qn * B1 * (int64_t)cs < ((int64_t)1 << 31) - ((int64_t)1 << 20);
        b_lay = two ? LAY_CONTIG2 : LAY_CONTIG;
        b_lines = (int64_t)qn * (dcny > 0 ? Bd.Rn - 1 : Bd.Rn);
      }
      HGP_TRY(run((int)(g.L[0] / 2), conv_mode, b_lay, Bd, b_lines));
      if (mid != nullptr) (*mid)(q0, qn, st);
      // C: INV along axis 1: column-major tiles -> row pairs, crop, fused dot or PCG update
      PassDesc Cd = base_desc();
      Cd.in = View{w1, B1, S0, 1, 0};
      Cd.out = View{yo, g.out_M, g.out[1], 1, (int)g.out[1]};
      Cd.dot = dvc; Cd.partial = pc;
      Cd.tw = g.tw[1].ptr; Cd.Q = qn; Cd.Rn = (int)((g.out[0] + 1) / 2); Cd.nrows = (int)g.out[0]; Cd.done = done;
      Cd.dcny = dcny;
      int epi_mode = EPI_OUT;
      if (epi != nullptr) {
        epi_mode = epi->mode;
        const int nrb = (Cd.Rn + rowt_pairs<T>((int)H1, 1) - 1) / rowt_pairs<T>((int)H1, 1);
        Cd.cg_r = reinterpret_cast<T*>(epi->r) + q0 * g.out_M;
        Cd.cg_x = reinterpret_cast<T*>(epi->x) + q0 * g.out_M;
        Cd.cg_p = reinterpret_cast<T*>(epi->p) + q0 * g.out_M;
        Cd.cg_coef = reinterpret_cast<const T*>(epi->coef) + q0;
        Cd.cg_part = epi->part ? reinterpret_cast<T*>(epi->part) + q0 * nrb : nullptr;
        set_cg_scalar<T>(Cd, epi, q0);
      }
      if (pair == nullptr) {
        HGP_TRY(run_rowt(1, Cd, epi_mode));
      } else {
        // K's row inverse also leaves the forward row transform of the new r in w1 (EPI_RF);
        // the chained op (C^-1, same L_K grid) continues at its axis-0 pass on this stream
        HGP_TRY(run_rowt(1, Cd, EPI_RF));
        PassDesc B2 = Bd;
        B2.spec = pair->spec;
        B2.spart = pair->spart != nullptr ? reinterpret_cast<T*>(pair->spart) + q0 * (H1 + 1) : nullptr;
        B2.spart_mid = (int)(H1 / 2);
        HGP_TRY(run((int)(g.L[0] / 2), conv_mode, b_lay, B2, b_lines));
        if (pair->mid != nullptr) (*pair->mid)(q0, qn, st);
        PassDesc C2d = Cd;
        const RowEpi* e2 = pair->epi;
        const int nrb = (Cd.Rn + rowt_pairs<T>((int)H1, 1) - 1) / rowt_pairs<T>((int)H1, 1);
        C2d.dot = nullptr; C2d.partial = nullptr;
        C2d.cg_r = reinterpret_cast<T*>(e2->r) + q0 * g.out_M;
        C2d.cg_x = reinterpret_cast<T*>(e2->x) + q0 * g.out_M;
        C2d.cg_p = reinterpret_cast<T*>(e2->p) + q0 * g.out_M;
        C2d.cg_coef = reinterpret_cast<const T*>(e2->coef) + q0;
        C2d.cg_part = e2->part ? reinterpret_cast<T*>(e2->part) + q0 * nrb : nullptr;
        C2d.cg_sp = nullptr; C2d.cg_np = 0; C2d.cg_rs = nullptr; C2d.cg_rs_out = nullptr;
        set_cg_scalar<T>(C2d, e2, q0);
        HGP_TRY(run_rowt(1, C2d, e2->mode));
      }
    } else if (d == 3 && !gen3) {
      C2<T>* w1 = reinterpret_cast<C2<T>*>(P->ws1.ptr) + (int64_t)slot * Qc * B1;
      C2<T>* w2 = reinterpret_cast<C2<T>*>(P->ws2.ptr) + (int64_t)slot * Qc * B2;
      const int64_t L1 = g.L[1], H2 = g.L[2] / 2, NC2 = H2 + 1, plane = NC2 * S1;
      auto run_rowt = [&](int inv, PassDesc& D, int epi_mode) -> int {
        const int me = pass_no++;
        if (only_pass >= 0 && only_pass != me) return 0;
        hipError_t e = launch_rowt<T>((int)H2, inv, epi_mode, D, st, 0);
        if (e != hipSuccess) return fail(HGP_E_HIP, std::string("3-D row pass launch: ") + hipGetErrorString(e));
        return 0;
      };
      auto run_linet = [&](int inv, PassDesc& D) -> int {
        const int me = pass_no++;
        if (only_pass >= 0 && only_pass != me) return 0;
        hipError_t e = launch_linet<T>((int)(L1 / 2), inv, D, st);
        if (e != hipSuccess) return fail(HGP_E_HIP, std::string("3-D line pass launch: ") + hipGetErrorString(e));
        return 0;
      };
      // Q1: FWD axis 2 on the row pairs of every (RHS, i0) plane -> w1 [q][i0][c2][i1]
      PassDesc A = base_desc();
      A.in = View{(void*)xi, g.in[1] * g.in[2], g.in[2], 1, (int)g.in[2]};
      A.out = View{w1, plane, S1, 1, 0};
      A.tw = g.tw[2].ptr; A.Q = (int)(qn * g.in[0]); A.Rn = (int)((g.in[1] + 1) / 2); A.nrows = (int)g.in[1];
      A.done = done;
      HGP_TRY(run_rowt(0, A, EPI_OUT));
      // Q2: FWD axis 1 (lines (i0, c2), i1 contiguous), transposed out -> w2 [q][c2][k1][i0]
      PassDesc Bd = base_desc();
      Bd.in = View{w1, g.in[0] * plane, S1, plane, (int)g.in[1]};
      Bd.out = View{w2, B2, L1 * S0, S0, (int)L1};
      Bd.tw = g.tw[1].ptr; Bd.Q = qn; Bd.Rn = (int)NC2; Bd.In = (int)g.in[0]; Bd.done = done;
      HGP_TRY(run_linet(0, Bd));
      // Q3: CONV axis 0 = contiguous lines (q, c2, k1), in place; spectrum [c2][k1][k0];
      // optional spectral dots spart [q][c2 * L1 + k1]
      PassDesc Cd = base_desc();
      Cd.in = View{w2, B2, S0, 1, (int)g.in[0]};
      Cd.out = View{w2, B2, S0, 1, (int)g.out[0]};
      Cd.spec = g.spec; Cd.spec_kind = g.spec_kind; Cd.spec_i = 0; Cd.spec_p = 1; Cd.spec_r = g.L[0];
      Cd.tw = g.tw[0].ptr; Cd.Q = qn; Cd.Rn = (int)(NC2 * L1); Cd.In = 1; Cd.done = done;
      if (spart != nullptr) {
        Cd.spart = reinterpret_cast<T*>(spart) + q0 * NC2 * L1;
        Cd.spart_mid = (int)(H2 / 2);
        Cd.spart_div = (int)L1;
      }
      HGP_TRY(run((int)(g.L[0] / 2), conv_mode, LAY_CONTIG, Cd, (int64_t)qn * Cd.Rn));
      if (mid != nullptr) (*mid)(q0, qn, st);
      // Q4: INV axis 1: w2 tiles -> lines (o0, c2), crop -> w1 [q][o0][c2][o1]
      PassDesc Dd = base_desc();
      Dd.in = View{w2, B2, L1 * S0, S0, (int)L1};
      Dd.out = View{w1, g.out[0] * plane, S1, plane, (int)g.out[1]};
      Dd.tw = g.tw[1].ptr; Dd.Q = qn; Dd.Rn = (int)NC2; Dd.In = (int)g.out[0]; Dd.done = done;
      HGP_TRY(run_linet(1, Dd));
      // Q5: INV axis 2 per (RHS, o0) plane: column-major tiles -> real rows, fused dot / PCG update
      PassDesc E = base_desc();
      E.in = View{w1, plane, S1, 1, 0};
      E.out = View{yo, g.out[1] * g.out[2], g.out[2], 1, (int)g.out[2]};
      E.dot = dvc; E.partial = pc;
      E.tw = g.tw[2].ptr; E.Q = (int)(qn * g.out[0]); E.Rn = (int)((g.out[1] + 1) / 2); E.nrows = (int)g.out[1];
      E.done = done;
      int epi_mode = EPI_OUT;
      if (epi != nullptr) {
        epi_mode = epi->mode;
        const int nrb = (E.Rn + rowt_pairs<T>((int)H2, 0) - 1) / rowt_pairs<T>((int)H2, 0);
        E.cg_r = reinterpret_cast<T*>(epi->r) + q0 * g.out_M;
        E.cg_x = reinterpret_cast<T*>(epi->x) + q0 * g.out_M;
        E.cg_p = reinterpret_cast<T*>(epi->p) + q0 * g.out_M;
        E.cg_coef = reinterpret_cast<const T*>(epi->coef) + q0;
        E.cg_div = (int)g.out[0];                 // planes per RHS share one alpha / beta
        E.cg_part = epi->part ? reinterpret_cast<T*>(epi->part) + q0 * g.out[0] * nrb : nullptr;
        set_cg_scalar<T>(E, epi, q0);
      }
      HGP_TRY(run_rowt(1, E, epi_mode));
    } else {
      C2<T>* w1 = reinterpret_cast<C2<T>*>(P->ws1.ptr) + (int64_t)slot * Qc * B1;
      C2<T>* w2 = reinterpret_cast<C2<T>*>(P->ws2.ptr) + (int64_t)slot * Qc * B2;
      const int64_t L1 = g.L[1], H2 = g.L[2] / 2;
      const int64_t rows_in = g.in[0] * g.in[1];
      // P1: FWD axis 2, row pairs -> w1 [q][i0][i1][c2]
      PassDesc P1 = base_desc();
      P1.in = View{(void*)xi, g.in_M, g.in[2], 1, (int)g.in[2]};
      P1.out = View{w1, B1, Sl, 1, 0};
      P1.tw = g.tw[2].ptr; P1.Q = qn; P1.Rn = (int)((rows_in + 1) / 2); P1.nrows = (int)rows_in; P1.done = done;
      HGP_TRY(run((int)H2, PASS_FWD, LAY_RP, P1, (int64_t)qn * P1.Rn));
      // P2: FWD axis 1 (strided): lines (i0, c2) -> w2 [q][i0][k1][c2]
      PassDesc P2 = base_desc();
      P2.in = View{w1, B1, g.in[1] * Sl, Sl, (int)g.in[1]};
      P2.out = View{w2, B2, L1 * Sl, Sl, (int)L1};
      P2.tw = g.tw[1].ptr; P2.Q = qn; P2.Rn = (int)g.in[0]; P2.In = (int)(H2 + 1); P2.done = done;
      HGP_TRY(run((int)(L1 / 2), PASS_FWD, LAY_STRIDED, P2, 0));
      // P3: CONV axis 0 (strided, in place): lines (k1, c2)
      PassDesc P3 = base_desc();
      P3.in = View{w2, B2, Sl, L1 * Sl, (int)g.in[0]};
      P3.out = View{w2, B2, Sl, L1 * Sl, (int)g.out[0]};
      P3.spec = g.spec; P3.spec_kind = g.spec_kind; P3.spec_i = L1 * g.L[0]; P3.spec_r = g.L[0]; P3.spec_p = 1;
      P3.tw = g.tw[0].ptr; P3.Q = qn; P3.Rn = (int)L1; P3.In = (int)(H2 + 1); P3.done = done;
      HGP_TRY(run((int)(g.L[0] / 2), conv_mode, LAY_STRIDED, P3, 0));
      // P4: INV axis 1 (strided): lines (o0, c2) -> w1 [q][o0][o1][c2]
      PassDesc P4 = base_desc();
      P4.in = View{w2, B2, L1 * Sl, Sl, (int)L1};
      P4.out = View{w1, B1, g.out[1] * Sl, Sl, (int)g.out[1]};
      P4.tw = g.tw[1].ptr; P4.Q = qn; P4.Rn = (int)g.out[0]; P4.In = (int)(H2 + 1); P4.done = done;
      HGP_TRY(run((int)(L1 / 2), PASS_INV, LAY_STRIDED, P4, 0));
      // P5: INV axis 2: rebuild row pairs, crop, fused dot
      PassDesc P5 = base_desc();
      P5.in = View{w1, B1, Sl, 1, (int)g.L[2]};
      P5.out = View{yo, g.out_M, g.out[2], 1, (int)g.out[2]};
      P5.dot = dvc; P5.partial = pc;
      P5.tw = g.tw[2].ptr; P5.Q = qn; P5.Rn = (int)((rows_out + 1) / 2); P5.nrows = (int)rows_out; P5.done = done;
      HGP_TRY(run((int)H2, PASS_INV, LAY_RP, P5, (int64_t)qn * P5.Rn));
    }
  }
  for (int i = 1; i < NS; ++i) {   // join: later work on the plan's stream sees every chunk
    HIP_TRY(hipEventRecord(P->ev_join[i - 1], streams[i]));
    HIP_TRY(hipStreamWaitEvent(P->stream, P->ev_join[i - 1], 0));
  }
  return 0;
}

// Forward fp64 FFT of length L along lines r < Rn (stride r_stride) x inner lines i < In
// (adjacent), positions at stride ps, output in the pass order (index half*L/2 + k = frequency
// 2k + half).  Lines of L/2 <= 8192 points are one k_pass (a -> b).  Longer ones (the L_R = 32768
// of an axis of 4098..8192 points, and every axis beyond 8192 points) take radix-2 steps, as
// deep as needed: the two interleaved half-length subsequences (stride 2 ps) are transformed
// the same way, then k_r2_combine merges them into the pass order of the full length.  Every
// level moves its lines between the two buffers, so the result may end in either: *result.
// tw = W_L; lev[j] = W_{L / 2^(j+1)} (the plan's tw64Kl / tw64Rl of the axis).
int fft_lines_f64(hgp_plan* P, double2* a, double2* b, int64_t L, int64_t Rn, int64_t r_stride, int64_t In,
                  int64_t ps, const void* tw, const DevBuf* lev, int depth, double2** result,
                  const int* done = nullptr) {
  hipStream_t s = P->stream;
  if (L / 2 <= 8192) {
    PassDesc D = base_desc();
    D.done = done;
    D.in = View{a, 0, r_stride, ps, (int)L};
    D.out = View{b, 0, r_stride, ps, (int)L};
    D.tw = tw; D.Q = 1; D.Rn = (int)Rn; D.In = (int)In;
    if (ps == 1 && In == 1) HGP_TRY(launch<double>((int)(L / 2), PASS_FWD, LAY_CONTIG, D, Rn, s));
    else HGP_TRY(launch<double>((int)(L / 2), PASS_FWD, LAY_STRIDED, D, 0, s));
    *result = b;
    return 0;
  }
  if (lev == nullptr || depth >= hgp_plan::NLEV || lev[depth].ptr == nullptr || L % 4 != 0)
    return fail(HGP_E_UNSUPPORTED, "fp64 transform of " + std::to_string(L) + " points: no radix-2 twiddle level");
  double2* half_res = nullptr;
  for (int e = 0; e < 2; ++e) {
    double2* r = nullptr;
    HGP_TRY(fft_lines_f64(P, a + e * ps, b + e * ps, L / 2, Rn, r_stride, In, 2 * ps, lev[depth].ptr, lev, depth + 1, &r,
                          done));
    half_res = (r == a + e * ps) ? a : b;
  }
  double2* dst = (half_res == a) ? b : a;
  r2_combine(half_res, dst, L, Rn, r_stride, In, ps, reinterpret_cast<const double2*>(tw), s, done);
  HIP_TRY(hipGetLastError());
  *result = dst;
  return 0;
}

// the radix-2 twiddle levels matching an axis twiddle table of the plan (nullptr: none)
const DevBuf* tw_levels(const hgp_plan* P, const DevBuf* tw64, int ax) {
  if (tw64 == P->tw64R) return P->tw64Rl[ax];
  if (tw64 == P->tw64K) return P->tw64Kl[ax];
  return nullptr;
}

// Forward FFT of a full (unpruned) fp64 complex L-grid: a -> result pointer (a or b).
int fwd_grid_f64(hgp_plan* P, const int64_t* L, const DevBuf* tw64, double2* a, double2* b, double2** result,
                 const int* done) {
  const int d = P->d;
  double2* cur = a;
  double2* oth = b;
  auto step = [&](int ax, int64_t Rn, int64_t rs, int64_t In, int64_t ps) -> int {
    double2* r = nullptr;
    HGP_TRY(fft_lines_f64(P, cur, oth, L[ax], Rn, rs, In, ps, tw64[ax].ptr, tw_levels(P, tw64, ax), 0, &r, done));
    if (r != cur) std::swap(cur, oth);
    return 0;
  };
  if (d == 1) {
    HGP_TRY(step(0, 1, L[0], 1, 1));
  } else if (d == 2) {
    HGP_TRY(step(1, L[0], L[1], 1, 1));
    HGP_TRY(step(0, 1, 0, L[1], L[1]));
  } else {
    HGP_TRY(step(2, L[0] * L[1], L[2], 1, 1));
    HGP_TRY(step(1, L[0], L[1] * L[2], L[2], L[2]));
    HGP_TRY(step(0, 1, 0, L[1] * L[2], L[1] * L[2]));
  }
  *result = cur;
  return 0;
}

// Forward FFT of a REAL fp64 L-grid (d >= 2) that only needs the compact half spectrum of the
// last axis (the R filter): real row pairs -> compact half spectra (k_pass RP, pitch S), then
// the other axes over the H + 1 compact columns only, in place.  Result: b [k0][k1][S].
int fwd_grid_real_f64(hgp_plan* P, const int64_t* L, const DevBuf* tw64, const double* a, double2* b, int64_t S) {
  const int d = P->d;
  hipStream_t s = P->stream;
  const int64_t Ll = L[d - 1], H = Ll / 2;
  int64_t rows = 1;
  for (int ax = 0; ax < d - 1; ++ax) rows *= L[ax];
  PassDesc A = base_desc();     // last axis: real row pairs (fold: rows of length 2H)
  A.in = View{const_cast<double*>(a), 0, Ll, 1, (int)Ll};
  A.out = View{b, 0, S, 1, 0};
  A.tw = tw64[d - 1].ptr; A.Q = 1; A.Rn = (int)((rows + 1) / 2); A.nrows = (int)rows; A.In = 1;
  HGP_TRY(launch<double>((int)H, PASS_FWD, LAY_RP, A, A.Rn, s));
  if (d == 3) {                 // axis 1 (strided, in place): lines (k0, c)
    PassDesc Bd = base_desc();
    Bd.in = View{b, 0, L[1] * S, S, (int)L[1]};
    Bd.out = View{b, 0, L[1] * S, S, (int)L[1]};
    Bd.tw = tw64[1].ptr; Bd.Q = 1; Bd.Rn = (int)L[0]; Bd.In = (int)(H + 1);
    HGP_TRY(launch<double>((int)(L[1] / 2), PASS_FWD, LAY_STRIDED, Bd, 0, s));
  }
  PassDesc Cd = base_desc();    // axis 0 (strided, in place): lines (k1, c)
  const int64_t ps = (d == 3 ? L[1] : 1) * S;
  Cd.in = View{b, 0, S, ps, (int)L[0]};
  Cd.out = View{b, 0, S, ps, (int)L[0]};
  Cd.tw = tw64[0].ptr; Cd.Q = 1; Cd.Rn = (int)(d == 3 ? L[1] : 1); Cd.In = (int)(H + 1);
  HGP_TRY(launch<double>((int)(L[0] / 2), PASS_FWD, LAY_STRIDED, Cd, 0, s));
  return 0;
}

template <typename T>
int upload_twiddles(DevBuf& buf, int64_t L) {
  std::vector<T> h((size_t)(2 * L));
  for (int64_t q = 0; q < L; ++q) {
    const double ang = -2.0 * M_PI * (double)q / (double)L;
    h[2 * q] = (T)std::cos(ang);
    h[2 * q + 1] = (T)std::sin(ang);
  }
  HGP_TRY(buf.ensure(h.size() * sizeof(T)));
  HIP_TRY(hipMemcpy(buf.ptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

// Bluestein tables of axis `ax` (hgp_kernels.hip k_chirp_*): chirps on the m-grid and the
// chirp filter's spectrum on the operator length L_K (>= 2m - 1), scaled by 1/L_K so the
// CONVC pass's unnormalised inverse FFT returns the linear convolution.
int make_bluestein(hgp_plan* P, int ax) {
  hipStream_t s = P->stream;
  const int64_t m = P->m[ax], n = P->n[ax], L = P->LK[ax];
  HGP_TRY(P->bsPre[ax].ensure((size_t)m * sizeof(double2)));
  HGP_TRY(P->bsPost[ax].ensure((size_t)m * sizeof(double2)));
  HGP_TRY(P->bsFilt[ax].ensure((size_t)L * sizeof(double2)));
  chirp_tables(reinterpret_cast<double2*>(P->bsPre[ax].ptr), reinterpret_cast<double2*>(P->bsPost[ax].ptr), m, n, s);
  DevBuf h;
  HGP_TRY(h.ensure((size_t)L * sizeof(double2)));
  chirp_filter(reinterpret_cast<double2*>(h.ptr), m, n, L, 1.0 / (double)L, s);
  int rc = 0;
  if (L / 2 <= 8192) {
    PassDesc D = base_desc();
    D.in = View{h.ptr, L, L, 1, (int)L};
    D.out = View{P->bsFilt[ax].ptr, L, L, 1, (int)L};
    D.tw = P->tw64K[ax].ptr; D.Q = 1; D.Rn = 1; D.In = 1;
    rc = launch<double>((int)(L / 2), PASS_FWD, LAY_CONTIG, D, 1, s);
  } else {           // an axis of more than 8192 points: the radix-2 levels (pass order as above)
    double2* hp = reinterpret_cast<double2*>(h.ptr);
    double2* fp = reinterpret_cast<double2*>(P->bsFilt[ax].ptr);
    double2* r = nullptr;
    rc = fft_lines_f64(P, hp, fp, L, 1, L, 1, 1, P->tw64K[ax].ptr, P->tw64Kl[ax], 0, &r);
    if (rc == 0 && r != fp && hipMemcpyAsync(fp, r, (size_t)L * sizeof(double2), hipMemcpyDeviceToDevice, s) != hipSuccess)
      rc = fail(HGP_E_HIP, "bluestein filter copy");
  }
  if (rc == 0 && hipStreamSynchronize(s) != hipSuccess) rc = fail(HGP_E_HIP, "bluestein filter FFT");
  h.release();
  return rc;
}

// y = scale * DCT-I_n(x) along axis ax for `nb` stacked m-grids (in, out real fp64, [nb][M]):
// y[k] = scale * (x_0 + (-1)^k x_{m-1} + 2 sum_{0<t<m-1} x_t cos(2 pi t k / n)).
// Chirp pre-multiply -> CONVC pass along the axis (contiguous last axis, strided otherwise)
// -> chirp post-multiply and real part.  O(M log m) instead of a dense m x m product.
int dct_axis(hgp_plan* P, int ax, const double* in, double* out, int nb, double scale) {
  hipStream_t s = P->stream;
  const int64_t m = P->m[ax], L = P->LK[ax], total = nb * P->M;
  int64_t I = 1;
  for (int c = ax + 1; c < P->d; ++c) I *= P->m[c];
  const int64_t O = total / (m * I);
  HGP_TRY(P->setC.ensure((size_t)(3 * P->M) * sizeof(double2)));
  double2* c = reinterpret_cast<double2*>(P->setC.ptr);
  const double2* pre = reinterpret_cast<const double2*>(P->bsPre[ax].ptr);
  const double2* post = reinterpret_cast<const double2*>(P->bsPost[ax].ptr);
  chirp_pre(in, pre, c, total, m, I, s);
  if (L / 2 > 8192) {
    // an axis of more than 8192 points: the Bluestein convolution as forward transform (radix-2
    // levels, pass order), x filter (pass order), un-permuted to the natural order, and the
    // inverse as conj(FFT(conj .)) over [O][L][I] line batches
    DevBuf e1, e2;                   // freed after the stream sync below
    HGP_TRY(e1.ensure((size_t)(O * L * I) * sizeof(double2)));
    HGP_TRY(e2.ensure((size_t)(O * L * I) * sizeof(double2)));
    double2* E1 = reinterpret_cast<double2*>(e1.ptr);
    double2* E2 = reinterpret_cast<double2*>(e2.ptr);
    line_embed(c, E1, O, m, I, L, s);
    double2* X = nullptr;
    HGP_TRY(fft_lines_f64(P, E1, E2, L, O, L * I, I, I, P->tw64K[ax].ptr, P->tw64Kl[ax], 0, &X));
    double2* Z = X == E1 ? E2 : E1;
    line_mul_unperm_conj(X, reinterpret_cast<const double2*>(P->bsFilt[ax].ptr), Z, O, L, I, s);
    double2* Y = nullptr;
    HGP_TRY(fft_lines_f64(P, Z, X, L, O, L * I, I, I, P->tw64K[ax].ptr, P->tw64Kl[ax], 0, &Y));
    line_unperm_conj(Y, c, O, L, I, m, s);
    chirp_post(c, post, out, total, m, I, scale, s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
  }
  PassDesc D = base_desc();
  D.spec = P->bsFilt[ax].ptr; D.spec_kind = SPEC_CPLX; D.spec_i = 0; D.spec_r = 0; D.spec_p = 1;
  D.tw = P->tw64K[ax].ptr; D.Q = 1;
  if (I == 1) {
    D.in = View{c, 0, m, 1, (int)m};
    D.out = View{c, 0, m, 1, (int)m};
    D.Rn = (int)O; D.In = 1;
    HGP_TRY(launch<double>((int)(L / 2), PASS_CONVC, LAY_CONTIG, D, O, s));
  } else {
    D.in = View{c, 0, m * I, I, (int)m};
    D.out = View{c, 0, m * I, I, (int)m};
    D.Rn = (int)O; D.In = (int)I;
    HGP_TRY(launch<double>((int)(L / 2), PASS_CONVC, LAY_STRIDED, D, 0, s));
  }
  chirp_post(c, post, out, total, m, I, scale, s);
  HIP_TRY(hipGetLastError());
  return 0;
}

template <typename T>
int set_column_t(hgp_plan* P, const void* column, double jitter, double clamp_min, int64_t* n_clamped) {
  hipStream_t s = P->stream;
  const int d = P->d;
  const int64_t M = P->M;
  HGP_TRY(P->setM1.ensure(3 * M * sizeof(double)));
  HGP_TRY(P->setM2.ensure(3 * M * sizeof(double)));
  HGP_TRY(P->Dm3.ensure(3 * M * sizeof(double)));
  HGP_TRY(P->nclamp.ensure(3 * sizeof(unsigned long long)));   // count, max D, max 1/D (pack_scale)
  double* a = reinterpret_cast<double*>(P->setM1.ptr);
  double* b = reinterpret_cast<double*>(P->setM2.ptr);
  to_f64<T>(column, a, M, jitter, s);
  P->clamp_min = clamp_min;
  // D_raw = DCT-I over every axis (length-n FFT of the circulant embedding, real part)
  for (int ax = 0; ax < d; ++ax) {
    HGP_TRY(dct_axis(P, ax, a, b, 1, 1.0));
    std::swap(a, b);
  }
  HIP_TRY(hipMemsetAsync(P->nclamp.ptr, 0, 3 * sizeof(unsigned long long), s));
  double* D3 = reinterpret_cast<double*>(P->Dm3.ptr);
  GridDims gm;
  gm.d = d;
  for (int ax = 0; ax < 3; ++ax) { gm.m[ax] = P->m[ax]; gm.n[ax] = P->n[ax]; gm.L[ax] = P->LK[ax]; }
  clamp_spectrum(a, D3, M, clamp_min, reinterpret_cast<unsigned long long*>(P->nclamp.ptr), gm, s);
  // generators: c_K = IFFT_n(D), c_inv = IFFT_n(1/D), s = IFFT_n(sqrt D) on the m-grid
  double* src = D3;
  double* dst = a;
  for (int ax = 0; ax < d; ++ax) {
    HGP_TRY(dct_axis(P, ax, src, dst, 3, 1.0 / (double)P->n[ax]));
    src = dst;
    dst = (dst == a) ? b : a;
  }
  const double* cK = src;
  const double* cI = src + M;
  const double* sv = src + 2 * M;
  // operator spectra on the power-of-two grids
  // the compact R grid of fwd_grid_real_f64 has a last axis of compact_stride(L) >= L/2 + 1
  // columns, more than L itself when L = 4 (an axis of 2 points)
  const int64_t Lr_last = P->LR[d - 1];
  const int64_t big = std::max({P->prodLK, P->prodLR, P->prodLR / Lr_last * compact_stride(Lr_last)});
  HGP_TRY(P->set1.ensure((size_t)big * sizeof(double2)));
  HGP_TRY(P->set2.ensure((size_t)big * sizeof(double2)));
  double2* g1 = reinterpret_cast<double2*>(P->set1.ptr);
  double2* g2 = reinterpret_cast<double2*>(P->set2.ptr);
  GridDims gd;
  gd.d = d;
  for (int ax = 0; ax < 3; ++ax) { gd.m[ax] = P->m[ax]; gd.n[ax] = P->n[ax]; gd.L[ax] = P->LK[ax]; }
  // K real, C^-1 imaginary, the latter scaled to K's magnitude (pack_scale, hgp_internal.hpp)
  const unsigned long long* pmx = reinterpret_cast<const unsigned long long*>(P->nclamp.ptr) + 1;
  embed_K(cK, cI, g1, gd, pmx, s);
  double2* F = nullptr;
  HGP_TRY(fwd_grid_f64(P, P->LK, P->tw64K, g1, g2, &F));
  if (P->grid_k) {
    // K / C^-1 on the full grid: the packed transform itself (K real, C^-1 imaginary), / N
    HGP_TRY(P->specKg.ensure((size_t)P->prodLK * sizeof(double2)));
    scale_copy(F, reinterpret_cast<double2*>(P->specKg.ptr), P->prodLK, 1.0 / (double)P->prodLK, s, pmx);
  }
  const int compact = d > 1 ? 1 : 0;
  const int64_t LKl = P->LK[d - 1], LRl = P->LR[d - 1];
  const int64_t SK = compact ? compact_stride(LKl) : LKl, SR = compact ? compact_stride(LRl) : LRl;
  // 3-D: [c2][k1][k0] (c2 <= H2, no pitch padding), the contiguous axis-0 lines (q, c2, k1)
  const int64_t nK = d == 3 ? P->prodLK / LKl * (LKl / 2 + 1) : P->prodLK / LKl * SK;
  const int64_t nR = d == 3 ? P->prodLR / LRl * (LRl / 2 + 1) : P->prodLR / LRl * SR;
  if (!P->grid_k) {   // the pass spectra (grid_k plans run K / C^-1 on the full grid)
    HGP_TRY(P->specK.ensure((size_t)nK * sizeof(T)));
    HGP_TRY(P->specI.ensure((size_t)nK * sizeof(T)));
    // d >= 2: spectra transposed to [compact column][k1][k0] for the contiguous axis-0 pass
    if (d == 1)
      extract_pair<T>(F, P->specK.ptr, P->specI.ptr, nK, LKl, SK, compact, 1.0 / (double)P->prodLK, s, 0, 0, pmx);
    else
      extract_t<T>(F, P->specK.ptr, P->specI.ptr, P->LK[0], d == 3 ? P->LK[1] : 1, LKl / 2, LKl, 0,
                   1.0 / (double)P->prodLK, s, pmx);
  }
  for (int ax = 0; ax < 3; ++ax) gd.L[ax] = P->LR[ax];
  bool long_r = false;
  for (int ax = 0; ax < d; ++ax) long_r = long_r || P->LR[ax] / 2 > 8192;
  bool sym = d >= 2 && !long_r;
  for (int ax = 0; ax < d; ++ax) sym = sym && P->LR[ax] >= 2 * P->n[ax] - 1;
  P->r_real = sym && !P->grid_r;
  if (P->grid_r) {
    // R / R^T on the full grid only (run_op_grid): the complex transform in its stored order, / N
    embed_R(sv, g1, gd, s);
    HGP_TRY(fwd_grid_f64(P, P->LR, P->tw64R, g1, g2, &F));
    HGP_TRY(P->specRg.ensure((size_t)P->prodLR * sizeof(double2)));
    scale_copy(F, reinterpret_cast<double2*>(P->specRg.ptr), P->prodLR, 1.0 / (double)P->prodLR, s);
  } else if (d == 1) {
    HGP_TRY(P->specR.ensure((size_t)nR * sizeof(C2<T>)));
    embed_R(sv, g1, gd, s);
    HGP_TRY(fwd_grid_f64(P, P->LR, P->tw64R, g1, g2, &F));
    extract_cplx<T>(F, P->specR.ptr, nR, LRl, SR, compact, 1.0 / (double)P->prodLR, s);
  } else if (!long_r) {
    HGP_TRY(P->specR.ensure((size_t)nR * (sym ? sizeof(T) : sizeof(C2<T>))));
    // the R filter is real: real row-pair transform of the last axis, compact columns only after
    embed_R_real(sv, reinterpret_cast<double*>(g1), gd, sym ? 1 : 0, s);
    HGP_TRY(fwd_grid_real_f64(P, P->LR, P->tw64R, reinterpret_cast<const double*>(g1), g2, SR));
    if (sym)   // even filter: its spectrum is real (the imaginary parts are rounding noise)
      extract_t_re<T>(g2, P->specR.ptr, P->LR[0], d == 3 ? P->LR[1] : 1, LRl / 2, SR, 1,
                      1.0 / (double)P->prodLR, s);
    else
      extract_t<T>(g2, P->specR.ptr, nullptr, P->LR[0], d == 3 ? P->LR[1] : 1, LRl / 2, SR, 1,
                   1.0 / (double)P->prodLR, s);
  } else {
    // an axis of L_R > 16384 points (fp32 passes of 16384-point halves): the full complex grid
    // through fft_lines_f64's radix-2 step
    HGP_TRY(P->specR.ensure((size_t)nR * sizeof(C2<T>)));
    embed_R(sv, g1, gd, s);
    HGP_TRY(fwd_grid_f64(P, P->LR, P->tw64R, g1, g2, &F));
    extract_t<T>(F, P->specR.ptr, nullptr, P->LR[0], d == 3 ? P->LR[1] : 1, LRl / 2, LRl, 0,
                 1.0 / (double)P->prodLR, s);
  }
  HIP_TRY(hipGetLastError());
  P->have_spec = true;
  if (n_clamped) {
    unsigned long long h = 0;
    HIP_TRY(hipMemcpyAsync(&h, P->nclamp.ptr, sizeof(h), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *n_clamped = (int64_t)h;
  }
  return 0;
}

// ---- grid-block (slab) sharding along axis 0 (hipgp_amd/slab.py) ----------------------------
// The op's pass sequence split at its axis-0 convolution.  Exchange layout E (plan dtype, complex):
//   E[g][q][i][c]  g < NG: d = 2 the compact column of axis 1 (NG = L1/2 + 1, inner = 1);
//                          d = 3 the axis-1 frequency k1 (NG = L1, inner = compact stride of axis 2)
//                  q < nrhs, i: the axis-0 row (the rank's rows, or whole lines in CONV)
// so the groups a rank owns after the all-to-all are one contiguous block.
struct SlabGeom { int64_t NG, inner; };
SlabGeom slab_geom(const hgp_plan* P, int op) {
  const OpGeom g = op_geom(P, op);
  if (P->d == 2) return SlabGeom{g.L[1] / 2 + 1, 1};
  return SlabGeom{g.L[1], compact_stride(g.L[2])};
}

// the INV stage's fused dot: per-row-pair partials [q][Rn] -> dot_out[q] (fixed order)
template <typename T>
int slab_dot_parts(hgp_plan* P, PassDesc& D, const void* dotv, int64_t nrhs, int64_t Rn) {
  if (dotv == nullptr) return 0;
  HGP_TRY(P->slab_part.ensure((size_t)(nrhs * Rn) * sizeof(T)));
  D.dot = dotv;
  D.partial = P->slab_part.ptr;
  return 0;
}

template <typename T>
int slab_pass_t(hgp_plan* P, int op, int stage, const void* in, void* out, int64_t nrhs, int64_t nrows, int64_t g0,
                int64_t ng, const void* dotv, void* dot_out, const int* done) {
  if (grid_route(P, op))
    return fail(HGP_E_UNSUPPORTED, "grid-block sharding of an operator on the full-grid route (fp64 lines of "
                                   "more than 16384 points, or an axis of more than 8192 points)");
  const OpGeom g = op_geom(P, op);
  const int d = P->d;
  const SlabGeom sg = slab_geom(P, op);
  const int conv_mode = g.spec_kind == SPEC_REAL ? PASS_CONV : PASS_CONVC;
  hipStream_t st = P->stream;
  const size_t cs = sizeof(C2<T>);
  auto sbase = [&]() {      // every slab pass is skipped once the slab PCG's device flag is set
    PassDesc D = base_desc();
    D.done = done;
    return D;
  };
  auto rowt = [&](int inv, PassDesc& D, int64_t H) -> int {
    hipError_t e = launch_rowt<T>((int)H, inv, EPI_OUT, D, st, 0);
    if (e == hipErrorNotSupported)
      return fail(HGP_E_UNSUPPORTED, "row transform of H = " + std::to_string(H) + " points does not fit one CU's LDS");
    if (e != hipSuccess) return fail(HGP_E_HIP, std::string("slab row pass: ") + hipGetErrorString(e));
    return 0;
  };
  const int64_t rows_len = stage == HGP_SLAB_FWD ? g.in[0] : g.out[0];
  const bool conv = stage == HGP_SLAB_CONV || stage == HGP_SLAB_CONV_A2A;
  if (!conv && (nrows < 1 || nrows > rows_len))
    return fail(HGP_E_ARG, "nrows must be in [1, " + std::to_string(rows_len) + "]");
  if (conv && (g0 < 0 || ng < 1 || g0 + ng > sg.NG))
    return fail(HGP_E_ARG, "groups [g0, g0 + ng) must lie in [0, " + std::to_string(sg.NG) + ")");
  if (stage == HGP_SLAB_CONV_A2A) {
    // rank-block layouts of the two all-to-all buffers (hgp_pass.hpp LAY_SEG_*): nrows = ranks
    if (nrows < 1) return fail(HGP_E_ARG, "HGP_SLAB_CONV_A2A: nrows is the world size (>= 1)");
    if (in == out) return fail(HGP_E_ARG, "HGP_SLAB_CONV_A2A: in and out must differ");
    const int64_t inner = d == 2 ? 1 : sg.inner;
    const int64_t P0 = std::max(g.in[0], g.out[0]);
    if (ng * nrhs * P0 * inner >= ((int64_t)1 << 31)) return fail(HGP_E_UNSUPPORTED, "slab too large");
    PassDesc Sd = sbase();
    Sd.in = View{const_cast<void*>(in), 0, 0, inner, (int)g.in[0]};
    Sd.out = View{out, 0, 0, inner, (int)g.out[0]};
    Sd.seg_ws = (int)nrows;
    const size_t se = g.spec_kind == SPEC_REAL ? sizeof(T) : cs;
    Sd.spec = static_cast<const char*>(g.spec) + (size_t)(g0 * g.L[0]) * se;
    Sd.spec_kind = g.spec_kind; Sd.spec_p = 1; Sd.spec_r = g.L[0];
    Sd.tw = g.tw[0].ptr; Sd.Q = (int)nrhs; Sd.Rn = (int)ng;
    if (d == 2) {     // lines (g, q), position-fast; spectrum [c1][k0]
      Sd.spec_i = 0; Sd.In = 1;
      return launch<T>((int)(g.L[0] / 2), conv_mode, LAY_SEG_C, Sd, nrhs * ng, st);
    }
    // d = 3: lines (g = k1, q) x c2 (adjacent); spectrum [c2][k1][k0]
    Sd.spec_i = g.L[1] * g.L[0]; Sd.In = (int)(g.L[2] / 2 + 1);
    return launch<T>((int)(g.L[0] / 2), conv_mode, LAY_SEG_S, Sd, 0, st);
  }
  if (d == 2) {
    const int64_t H1 = g.L[1] / 2;
    if (stage == HGP_SLAB_FWD || stage == HGP_SLAB_INV) {
      // the row kernels address one RHS's columns with 32-bit byte offsets from its base
      if (sg.NG * nrhs * nrows * (int64_t)cs >= ((int64_t)1 << 31))
        return fail(HGP_E_UNSUPPORTED, "slab too large: NG * nrhs * nrows complex values exceed 2 GiB");
      PassDesc D = sbase();
      D.tw = g.tw[1].ptr; D.Q = (int)nrhs; D.Rn = (int)((nrows + 1) / 2); D.nrows = (int)nrows;
      if (stage == HGP_SLAB_FWD) {
        D.in = View{const_cast<void*>(in), nrows * g.in[1], g.in[1], 1, (int)g.in[1]};
        D.out = View{out, nrows, nrhs * nrows, 1, 0};
        return rowt(0, D, H1);
      }
      D.in = View{const_cast<void*>(in), nrows, nrhs * nrows, 1, 0};
      D.out = View{out, nrows * g.out[1], g.out[1], 1, (int)g.out[1]};
      HGP_TRY(slab_dot_parts<T>(P, D, dotv, nrhs, D.Rn));
      HGP_TRY(rowt(1, D, H1));
      if (dotv != nullptr) reduce_rows<T>(D.partial, D.Rn, (int)nrhs, dot_out, st);
      return 0;
    }
    if (stage != HGP_SLAB_CONV) return fail(HGP_E_ARG, "bad slab stage");
    const int64_t P0 = std::max(g.in[0], g.out[0]);
    PassDesc Bd = sbase();
    Bd.in = View{const_cast<void*>(in), P0, nrhs * P0, 1, (int)g.in[0]};
    Bd.out = View{out, P0, nrhs * P0, 1, (int)g.out[0]};
    const size_t se = g.spec_kind == SPEC_REAL ? sizeof(T) : cs;
    Bd.spec = static_cast<const char*>(g.spec) + (size_t)(g0 * g.L[0]) * se;
    Bd.spec_kind = g.spec_kind; Bd.spec_i = 0; Bd.spec_p = 1; Bd.spec_r = g.L[0];
    Bd.tw = g.tw[0].ptr; Bd.Q = (int)nrhs; Bd.Rn = (int)ng; Bd.In = 1;
    return launch<T>((int)(g.L[0] / 2), conv_mode, LAY_CONTIG, Bd, nrhs * ng, st);
  }
  // d = 3
  const int64_t Sl = sg.inner, L1 = g.L[1], H2 = g.L[2] / 2;
  if (stage == HGP_SLAB_FWD || stage == HGP_SLAB_INV) {
    const int64_t r1 = stage == HGP_SLAB_FWD ? g.in[1] : g.out[1];
    const int64_t wsz = nrhs * nrows * r1 * Sl;
    if (L1 * nrhs * nrows * Sl >= ((int64_t)1 << 31) || wsz >= ((int64_t)1 << 31))
      return fail(HGP_E_UNSUPPORTED, "slab too large for 32-bit element offsets");
    HGP_TRY(P->ws1.ensure((size_t)wsz * cs));
    C2<T>* w1 = reinterpret_cast<C2<T>*>(P->ws1.ptr);
    if (stage == HGP_SLAB_FWD) {
      PassDesc P1 = sbase();   // axis 2: real row pairs -> w1 [q][i][i1][c2]
      P1.in = View{const_cast<void*>(in), nrows * g.in[1] * g.in[2], g.in[2], 1, (int)g.in[2]};
      P1.out = View{w1, nrows * r1 * Sl, Sl, 1, 0};
      P1.tw = g.tw[2].ptr; P1.Q = (int)nrhs; P1.Rn = (int)((nrows * r1 + 1) / 2); P1.nrows = (int)(nrows * r1);
      HGP_TRY(launch<T>((int)H2, PASS_FWD, LAY_RP, P1, nrhs * P1.Rn, st));
      PassDesc P2 = sbase();   // axis 1 (strided): w1 -> E [k1][q][i][c2]
      P2.in = View{w1, nrows * r1 * Sl, r1 * Sl, Sl, (int)r1};
      P2.out = View{out, nrows * Sl, Sl, nrhs * nrows * Sl, (int)L1};
      P2.tw = g.tw[1].ptr; P2.Q = (int)nrhs; P2.Rn = (int)nrows; P2.In = (int)(H2 + 1);
      return launch<T>((int)(L1 / 2), PASS_FWD, LAY_STRIDED, P2, 0, st);
    }
    PassDesc P4 = sbase();     // axis 1 inverse (strided): E [k1][q][o][c2] -> w1 [q][o][o1][c2]
    P4.in = View{const_cast<void*>(in), nrows * Sl, Sl, nrhs * nrows * Sl, (int)L1};
    P4.out = View{w1, nrows * r1 * Sl, r1 * Sl, Sl, (int)r1};
    P4.tw = g.tw[1].ptr; P4.Q = (int)nrhs; P4.Rn = (int)nrows; P4.In = (int)(H2 + 1);
    HGP_TRY(launch<T>((int)(L1 / 2), PASS_INV, LAY_STRIDED, P4, 0, st));
    PassDesc P5 = sbase();     // axis 2 inverse: w1 -> real rows (crop)
    P5.in = View{w1, nrows * r1 * Sl, Sl, 1, (int)g.L[2]};
    P5.out = View{out, nrows * r1 * g.out[2], g.out[2], 1, (int)g.out[2]};
    P5.tw = g.tw[2].ptr; P5.Q = (int)nrhs; P5.Rn = (int)((nrows * r1 + 1) / 2); P5.nrows = (int)(nrows * r1);
    HGP_TRY(slab_dot_parts<T>(P, P5, dotv, nrhs, P5.Rn));
    HGP_TRY(launch<T>((int)H2, PASS_INV, LAY_RP, P5, nrhs * P5.Rn, st));
    if (dotv != nullptr) reduce_rows<T>(P5.partial, P5.Rn, (int)nrhs, dot_out, st);
    return 0;
  }
  if (stage != HGP_SLAB_CONV) return fail(HGP_E_ARG, "bad slab stage");
  const int64_t P0 = std::max(g.in[0], g.out[0]);
  if (ng * nrhs * P0 * Sl >= ((int64_t)1 << 31)) return fail(HGP_E_UNSUPPORTED, "slab too large for 32-bit element offsets");
  PassDesc P3 = sbase();       // axis 0 conv (strided over i), lines (k1, c2) of each RHS
  P3.in = View{const_cast<void*>(in), P0 * Sl, nrhs * P0 * Sl, Sl, (int)g.in[0]};
  P3.out = View{out, P0 * Sl, nrhs * P0 * Sl, Sl, (int)g.out[0]};
  const size_t se = g.spec_kind == SPEC_REAL ? sizeof(T) : cs;
  // spectrum [c2][k1][k0]: group g = k1, inner line = c2
  P3.spec = static_cast<const char*>(g.spec) + (size_t)(g0 * g.L[0]) * se;
  P3.spec_kind = g.spec_kind; P3.spec_i = L1 * g.L[0]; P3.spec_r = g.L[0]; P3.spec_p = 1;
  P3.tw = g.tw[0].ptr; P3.Q = (int)nrhs; P3.Rn = (int)ng; P3.In = (int)(H2 + 1);
  return launch<T>((int)(g.L[0] / 2), conv_mode, LAY_STRIDED, P3, 0, st);
}

// ---- PCG -------------------------------------------------------------------------------------
// the 3-D operators run their axis-2 rows through the row-pair kernels (per i0 plane) when
// those fit one CU's LDS; the dot partials then come per (plane, row pair)
template <typename T>
bool planes3d(const hgp_plan* P) {
  return P->d == 3 && rowt_fits<T>((int)(P->LK[2] / 2), 0) != 0 && linet_fits<T>((int)(P->LK[1] / 2)) != 0;
}
template <typename T>
int rn_last(const hgp_plan* P) {
  if (P->grid_k) return update_np(P->M);   // run_op_grid's rowdot partials
  if (P->d == 1) return 1;
  if (P->d == 2) return (int)((P->m[0] + 1) / 2);
  if (planes3d<T>(P)) return (int)(P->m[0] * ((P->m[1] + 1) / 2));
  return (int)((P->m[0] * P->m[1] + 1) / 2);
}

// Fused PCG (pcg_step_t): the dots p.Ap and z.r come from the axis-0 conv pass as spectral
// sums over its lines (2-D: per compact column c1, L_1/2 + 1 partials per RHS; 3-D: per (c2,
// k1), (L_2/2 + 1) L_1 partials); r.r from the fused x/r update, one partial per row block of
// the row-inverse pass (3-D: per block of each i0 plane).
int spec_np(const hgp_plan* P) {
  return P->d == 2 ? (int)(P->LK[1] / 2 + 1) : (int)((P->LK[2] / 2 + 1) * P->LK[1]);
}
// the fused PCG needs the row-pair kernels of the K / C^-1 rows
template <typename T>
bool fused_pcg(const hgp_plan* P) {
  if (P->grid_k) return false;
  return (P->d == 2 && rowt_fits<T>((int)(P->LK[1] / 2), 1) != 0) || planes3d<T>(P);
}
template <typename T>
int xr_np(const hgp_plan* P) {
  if (P->d == 2) {
    const int pairs = rowt_pairs<T>((int)(P->LK[1] / 2), 1);
    return (int)(((P->m[0] + 1) / 2 + pairs - 1) / pairs);
  }
  const int pairs = rowt_pairs<T>((int)(P->LK[2] / 2), 0);
  return (int)(P->m[0] * (((P->m[1] + 1) / 2 + pairs - 1) / pairs));
}

template <typename T>
int pcg_begin_t(hgp_plan* P, const void* b, void* x, int64_t nrhs, int use_precond, int layout) {
  hipStream_t s = P->stream;
  const int64_t M = P->M;
  const size_t vb = (size_t)(nrhs * M) * sizeof(T);
  const bool fused = fused_pcg<T>(P);
  HGP_TRY(P->r.ensure(vb));
  HGP_TRY(P->p.ensure(vb));
  // the fused iteration never stores Ap or z (the row-inverse epilogues consume them in LDS), so
  // only the unfused one holds them: at C4's B = 200 that is 27 GB of scratch less, and the
  // plan then fits the idle-pool budget instead of being trimmed and re-allocated per solve
  if (!fused) {
    HGP_TRY(P->z.ensure(vb));
    HGP_TRY(P->Ap.ensure(vb));
  }
  const int npo = fused ? std::max(rn_last<T>(P), spec_np(P)) : rn_last<T>(P);
  const int npu = fused ? std::max(update_np(M), xr_np<T>(P)) : update_np(M);
  HGP_TRY(P->part_op.ensure((size_t)(nrhs * npo) * sizeof(T)));
  HGP_TRY(P->part_u.ensure((size_t)(nrhs * npu) * sizeof(T)));
  if (fused && fold_groups(spec_np(P)) > 0) HGP_TRY(P->part_f.ensure((size_t)(nrhs * fold_groups(spec_np(P))) * sizeof(T)));
  HGP_TRY(P->scal.ensure((size_t)(5 * nrhs) * sizeof(T)));   // rs, alpha, beta, rnew, rs (2nd)
  HGP_TRY(P->flags.ensure(16));
  const void* brow = b;
  void* xrow = x;
  if (layout == HGP_LAYOUT_COLS) {
    HGP_TRY(P->bT.ensure(vb));
    HGP_TRY(P->xT.ensure(vb));
    transpose<T>(b, P->bT.ptr, M, nrhs, s);   // (M, nrhs) -> (nrhs, M)
    brow = P->bT.ptr;
    xrow = P->xT.ptr;
  }
  int* flags = reinterpret_cast<int*>(P->flags.ptr);
  HIP_TRY(hipMemsetAsync(flags, 0, 16, s));
  T* sc = reinterpret_cast<T*>(P->scal.ptr);
  T* rs = sc;
  cg_init<T>(brow, xrow, P->r.ptr, nrhs * M, s);
  if (use_precond && fused) {
    // p = z = C^-1 r straight into p; rs = z.r as the column pass's spectral dot
    HGP_TRY(run_op<T>(P, HGP_OP_CINV, P->r.ptr, P->p.ptr, nrhs, nullptr, nullptr, nullptr, -1, P->part_op.ptr));
    const int G = fold_groups(spec_np(P));
    if (G > 0) {
      fold_rows<T>(P->part_op.ptr, spec_np(P), (int)nrhs, P->part_f.ptr, nullptr, s);
      reduce_rows<T>(P->part_f.ptr, G, (int)nrhs, rs, s);
    } else {
      reduce_rows<T>(P->part_op.ptr, spec_np(P), (int)nrhs, rs, s);
    }
  } else if (use_precond) {
    HGP_TRY(run_op<T>(P, HGP_OP_CINV, P->r.ptr, P->z.ptr, nrhs, P->r.ptr, P->part_op.ptr, nullptr));
    reduce_rows<T>(P->part_op.ptr, npo, (int)nrhs, rs, s);
    vcopy<T>(P->z.ptr, P->p.ptr, nrhs * M, nullptr, s);
  } else {
    rowdot_part<T>(P->r.ptr, P->r.ptr, P->part_u.ptr, nrhs, M, npu, s);
    reduce_rows<T>(P->part_u.ptr, npu, (int)nrhs, rs, s);
    vcopy<T>(P->r.ptr, P->p.ptr, nrhs * M, nullptr, s);
  }
  HIP_TRY(hipGetLastError());
  P->cg_nrhs = nrhs;
  P->cg_precond = use_precond;
  P->cg_layout = layout;
  P->cg_x_user = x;
  P->cg_x = xrow;
  P->cg_rs_par = 0;
  P->cg_step = 0;
  P->cg_active = true;
  return 0;
}

template <typename T>
int pcg_step_t(hgp_plan* P, double tol) {
  hipStream_t s = P->stream;
  const int step = P->cg_step++;
  const int64_t nrhs = P->cg_nrhs, M = P->M;
  const int npo = rn_last<T>(P), npu = update_np(M);
  int* flags = reinterpret_cast<int*>(P->flags.ptr);
  int* done = flags;
  int* iters = flags + 1;
  T* sc = reinterpret_cast<T*>(P->scal.ptr);
  T* rs = sc;
  T* alpha = sc + nrhs;
  T* beta = sc + 2 * nrhs;
  T* rnew = sc + 3 * nrhs;
  if (fused_pcg<T>(P)) {
    // Fused iteration (2-D, 3-D).  K p: the axis-0 pass leaves the spectral p.Ap partials, from
    // which alpha is formed per RHS (in the row-inverse kernel, or by a small kernel between the
    // passes); the row-inverse epilogue does x += alpha p, r -= alpha Ap (+ r.r partials) with
    // Ap never stored.  Then the break test; then C^-1 r,
    // whose epilogue does p = z + beta p (z never stored).  Order and semantics of cg.py:63-78.
    const int nps0 = spec_np(P), npx = xr_np<T>(P);
    // alpha and beta are formed inside the row-inverse kernels (each block sums its RHS's
    // spectral partials, PassDesc::cg_sp) when the partials fit CG_LOADS per thread; rs then
    // alternates between two buffers (the beta epilogue writes the next one).  Otherwise
    // (long 3-D rows are folded per chunk first) k_cg_alpha / k_cg_beta run between the passes
    // of each chunk.
    // Reading the raw partials in every row-inverse block pays when they are a small share of
    // the block's tile (C2: 3 %, 15.9 -> 15.4 ms per PCG(20)).  C4's 4097 partials per 64-B
    // tile (6 %) measured 280 -> 285 ms, and folded partials (C4 after the fold, C5) +1 % / +-0,
    // so those keep the fold + small-kernel form.
    const int Hl = (int)(P->LK[P->d - 1] / 2);
    const int thr = rowt_threads<T>(Hl, P->d == 2);
    const int64_t tile_vals = 2 * (int64_t)(Hl + 1) * 2 * rowt_pairs<T>(Hl, P->d == 2);   // reals per block tile
    const bool direct = nps0 <= CG_LOADS * thr && 25 * (int64_t)nps0 <= tile_vals;
    const int G = direct ? 0 : fold_groups(nps0);
    const int nps = G > 0 ? G : nps0;
    const bool inkern = direct;
    T* part_o = reinterpret_cast<T*>(P->part_op.ptr);
    T* part_s = G > 0 ? reinterpret_cast<T*>(P->part_f.ptr) : part_o;
    auto fold = [&](int64_t q0, int qn, hipStream_t cs) {
      if (G > 0) fold_rows<T>(part_o + q0 * nps0, nps0, qn, part_s + q0 * G, done, cs);
    };
    T* rs_cur = P->cg_rs_par ? sc + 4 * nrhs : rs;
    T* rs_nxt = P->cg_rs_par ? rs : sc + 4 * nrhs;
    const MidFn mid_alpha = [&](int64_t q0, int qn, hipStream_t cs) {
      fold(q0, qn, cs);
      if (!inkern) cg_alpha<T>(part_s + q0 * nps, nps, qn, rs_cur + q0, alpha + q0, done, cs);
    };
    // with the preconditioner the x update moves to the C^-1 pass (EPI_R here, EPI_XP there)
    const bool defer = P->cg_precond != 0;
    RowEpi exr{defer ? EPI_R : EPI_XR, P->r.ptr, P->cg_x, P->p.ptr, alpha, P->part_u.ptr};
    if (inkern) { exr.sp = part_s; exr.np = nps; exr.rs = rs_cur; exr.alpha_out = alpha; }
    if (P->cg_precond && P->d == 2 && P->chain_pcg) {
      // 2-D: K p and C^-1 r chained per RHS chunk (run_op PairOp): K's row-inverse pass updates r
      // and leaves its forward row transform for C^-1 (EPI_RF), C^-1's row-inverse pass does
      // x += alpha p, p = z + beta p (EPI_XP); then the all-RHS break test.  The x update of the
      // iteration in which the break fires is the same either way, and the p update after it is
      // never read, so the C^-1 half no longer waits for the test (cg.py:67-75 arithmetic and
      // break rule unchanged; the fix-up pass of PassDesc::cg_fix is not needed).
      const MidFn mid_beta = [&](int64_t q0, int qn, hipStream_t cs) {
        fold(q0, qn, cs);
        if (!inkern) cg_beta<T>(part_s + q0 * nps, nps, qn, rs_cur + q0, beta + q0, done, cs);
      };
      RowEpi ep{EPI_XP, P->r.ptr, P->cg_x, P->p.ptr, beta, nullptr};
      ep.coef2 = alpha;
      ep.fix = -1;
      if (inkern) { ep.sp = part_s; ep.np = nps; ep.rs = rs_cur; ep.rs_out = rs_nxt; }
      const PairOp pair{P->specI.ptr, part_o, &ep, (G > 0 || !inkern) ? &mid_beta : nullptr};
      HGP_TRY(run_op<T>(P, HGP_OP_K, P->p.ptr, nullptr, nrhs, nullptr, nullptr, done, -1, part_o, &exr,
                        (G > 0 || !inkern) ? &mid_alpha : nullptr, &pair));
      cg_check<T>(P->part_u.ptr, npx, (int)nrhs, tol, rnew, done, iters, s);
      if (inkern) P->cg_rs_par ^= 1;
      HIP_TRY(hipGetLastError());
      return 0;
    }
    HGP_TRY(run_op<T>(P, HGP_OP_K, P->p.ptr, nullptr, nrhs, nullptr, nullptr, done, -1, part_o, &exr,
                      (G > 0 || !inkern) ? &mid_alpha : nullptr));
    cg_check<T>(P->part_u.ptr, npx, (int)nrhs, tol, rnew, done, iters, s);
    if (P->cg_precond) {
      const MidFn mid_beta = [&](int64_t q0, int qn, hipStream_t cs) {
        fold(q0, qn, cs);
        if (!inkern) cg_beta<T>(part_s + q0 * nps, nps, qn, rs_cur + q0, beta + q0, done, cs);
      };
      RowEpi ep{EPI_XP, P->r.ptr, P->cg_x, P->p.ptr, beta, nullptr};
      ep.coef2 = alpha;
      ep.fix = step + 1;           // the done value this step's break test writes
      if (inkern) { ep.sp = part_s; ep.np = nps; ep.rs = rs_cur; ep.rs_out = rs_nxt; }
      HGP_TRY(run_op<T>(P, HGP_OP_CINV, P->r.ptr, nullptr, nrhs, nullptr, nullptr, done, -1, part_o, &ep,
                        (G > 0 || !inkern) ? &mid_beta : nullptr));
      if (inkern) P->cg_rs_par ^= 1;
    } else {
      cg_beta<T>(P->part_u.ptr, npx, (int)nrhs, rs_cur, beta, done, s);
      cg_update_p<T>(P->p.ptr, P->r.ptr, beta, nrhs, M, done, s);
    }
    HIP_TRY(hipGetLastError());
    return 0;
  }
  // Ap = K p ; fused p.Ap
  HGP_TRY(run_op<T>(P, HGP_OP_K, P->p.ptr, P->Ap.ptr, nrhs, P->p.ptr, P->part_op.ptr, done));
  cg_alpha<T>(P->part_op.ptr, npo, (int)nrhs, rs, alpha, done, s);
  cg_update_xr<T>(P->cg_x, P->r.ptr, P->p.ptr, P->Ap.ptr, alpha, P->part_u.ptr, nrhs, M, done, s);
  cg_check<T>(P->part_u.ptr, npu, (int)nrhs, tol, rnew, done, iters, s);
  if (P->cg_precond) {
    HGP_TRY(run_op<T>(P, HGP_OP_CINV, P->r.ptr, P->z.ptr, nrhs, P->r.ptr, P->part_op.ptr, done));
    cg_beta<T>(P->part_op.ptr, npo, (int)nrhs, rs, beta, done, s);
    cg_update_p<T>(P->p.ptr, P->z.ptr, beta, nrhs, M, done, s);
  } else {
    cg_beta<T>(P->part_u.ptr, npu, (int)nrhs, rs, beta, done, s);
    cg_update_p<T>(P->p.ptr, P->r.ptr, beta, nrhs, M, done, s);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

template <typename T>
int pcg_finish_x(hgp_plan* P) {
  if (P->cg_layout == HGP_LAYOUT_COLS) transpose<T>(P->cg_x, P->cg_x_user, P->cg_nrhs, P->M, P->stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

#define DISPATCH(P, FN, ...) ((P)->dtype == HGP_F64 ? FN<double>(__VA_ARGS__) : FN<float>(__VA_ARGS__))

int check_plan(const hgp_plan* P) {
  if (P == nullptr) return fail(HGP_E_ARG, "null plan");
  return 0;
}

int use_device(const hgp_plan* P) {
  HIP_TRY(hipSetDevice(P->device));
  return 0;
}

}  // namespace

extern "C" {

const char* hgp_last_error(void) { return g_err.c_str(); }

const char* hgp_version(void) { return "hipgp-mi355x 0.1 (gfx950)"; }

int hgp_plan_create(int device, int ndim, const int64_t* m, int dtype, int64_t max_rhs, void* hip_stream,
                    hgp_plan** out) {
  if (out == nullptr || m == nullptr) return fail(HGP_E_ARG, "null argument");
  *out = nullptr;
  if (ndim < 1 || ndim > 3) return fail(HGP_E_ARG, "ndim must be 1..3 (torch.fft signal_ndim limit)");
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  (void)max_rhs;
  HIP_TRY(hipSetDevice(device));
  hgp_plan* P = new hgp_plan();
  P->device = device;
  P->dtype = dtype;
  P->stream = reinterpret_cast<hipStream_t>(hip_stream);
  P->esz = dtype == HGP_F64 ? 8 : 4;
  P->ndim_user = ndim;
  int d = 0;
  for (int a = 0; a < ndim; ++a) {
    if (m[a] < 1) { delete P; return fail(HGP_E_ARG, "grid sizes must be >= 1"); }
    if (m[a] == 1) continue;     // size-1 axes are identities (n = 1, hipgp.py:72)
    P->m[d] = m[a];
    P->n[d] = 2 * m[a] - 2;
    P->LK[d] = next_pow2(2 * m[a] - 1);
    P->LR[d] = next_pow2(4 * m[a] - 4);
    ++d;
  }
  P->d = d;
  // R / R^T length.  Exact for any L_R >= n + m - 1 = 3m - 3 per axis.  Default: the
  // power of two >= 2n, where the filter embeds evenly and the spectrum is real (r_real).  The
  // shortest admissible lengths -- 2^k or 3 * 2^k >= 3m - 3 -- take a complex spectrum instead;
  // they are used when their grid is below 0.6 of the real one's (a complex-spectrum point costs
  // more: C5's 768 x 768 x 384 is 0.42 of 1024 x 1024 x 512).  HGP_LR=pow2 keeps the default.
  {
    const char* lr = std::getenv("HGP_LR");
    const bool allow = !(lr && std::string(lr) == "pow2");
    double real_pts = 1, short_pts = 1;
    int64_t Ls[3] = {1, 1, 1};
    bool ok = allow && d >= 2;
    bool long_axis = false;
    for (int a = 0; a < d; ++a) {
      const int64_t need = 3 * P->m[a] - 3;
      Ls[a] = std::min(next_pow2(need), next_tri(need));
      real_pts *= (double)P->LR[a];
      short_pts *= (double)Ls[a];
      if (Ls[a] / 2 > 8192) ok = false;      // the fp64 set-up transforms hold L_R / 2 <= 8192
      long_axis = long_axis || P->m[a] > 8192;
    }
    if (ok && short_pts < 0.6 * real_pts)
      for (int a = 0; a < d; ++a) P->LR[a] = Ls[a];
    // an axis of more than 8192 points: every operator on the full fp64 grid (run_op_grid), whose
    // radix-2 levels take any L = 2^k or 3 * 2^k -- the shortest admissible L_R on every axis
    if (long_axis) {
      for (int a = 0; a < d; ++a) P->LR[a] = Ls[a];
      P->grid_k = P->grid_r = true;
    }
  }
  if (d == 0) { delete P; return fail(HGP_E_UNSUPPORTED, "a grid with every axis of size 1 (M = 1) is not supported"); }
  for (int a = 0; a < d; ++a) {
    // L_R / 2 = 16384 (axes of 4098..8192 points): fp32 operator passes hold one such line per
    // block; fp64 lines of 16384 points exceed one CU's LDS (the set-up's fp64 transforms of
    // them take fft_lines_f64's radix-2 step)
    if (!P->grid_k && (P->LR[a] / 2 > 16384 || P->LK[a] / 2 > 8192)) {
      delete P;
      return fail(HGP_E_UNSUPPORTED, "internal: pass lengths of a grid axis of at most 8192 points");
    }
    // fp64 lines of L_R / 2 > 8192 points exceed one CU's LDS: R / R^T take the full-grid route
    if (dtype == HGP_F64 && P->LR[a] / 2 > 8192) P->grid_r = true;
    P->M *= P->m[a];
    P->Mp *= P->n[a];
    P->prodLK *= P->LK[a];
    P->prodLR *= P->LR[a];
  }
  {
    size_t tot = 0;
    if (hipDeviceTotalMem(&tot, device) == hipSuccess && tot > 0)
      P->ws3_budget = std::max<int64_t>((int64_t)4 << 30, std::min<int64_t>(HGP_WS3_MAX, (int64_t)(tot / 8)));
  }
  const char* wb = std::getenv("HGP_WS_MB");
  if (wb) { P->ws_budget = (int64_t)std::atoll(wb) << 20; P->ws_explicit = true; }
  const char* hg = std::getenv("HGP_GRAPH");
  if (hg && std::atoi(hg) == 0) P->use_graphs = false;
  const char* ns = std::getenv("HGP_STREAMS");
  if (ns) P->nstreams = std::max(1, std::min(4, std::atoi(ns)));
  const char* cp = std::getenv("HGP_CHAIN_PCG");
  if (cp) P->chain_pcg = std::atoi(cp) != 0;
  const char* dn = std::getenv("HGP_DCNY");
  if (dn) P->dcny_pack = std::atoi(dn) != 0;
  const char* c32 = std::getenv("HGP_CONV_P32");
  if (c32) P->conv_p32 = std::atoi(c32) != 0;
  const char* bc = std::getenv("HGP_BALANCED_CHUNKS");
  if (bc) P->balanced_chunks = std::atoi(bc) != 0;
  int rc = 0;
  for (int a = 0; a < d && rc == 0; ++a) {
    if (dtype == HGP_F64) {
      rc = upload_twiddles<double>(P->twK[a], P->LK[a]);
      if (!rc) rc = upload_twiddles<double>(P->twR[a], P->LR[a]);
    } else {
      rc = upload_twiddles<float>(P->twK[a], P->LK[a]);
      if (!rc) rc = upload_twiddles<float>(P->twR[a], P->LR[a]);
    }
    if (!rc) rc = upload_twiddles<double>(P->tw64K[a], P->LK[a]);
    // W_{L/2}, W_{L/4}, ... for the radix-2 levels of lines longer than one fp64 pass
    for (int w = 0; w < 2 && !rc; ++w) {
      int64_t Lc = w == 0 ? P->LK[a] : P->LR[a];
      DevBuf* lev = w == 0 ? P->tw64Kl[a] : P->tw64Rl[a];
      for (int j = 0; Lc / 2 > 8192 && !rc; ++j) {
        if (j >= hgp_plan::NLEV) { rc = fail(HGP_E_UNSUPPORTED, "grid axis too long for the fp64 radix-2 levels"); break; }
        Lc /= 2;
        rc = upload_twiddles<double>(lev[j], Lc);
      }
    }
    if (!rc) rc = upload_twiddles<double>(P->tw64R[a], P->LR[a]);
    if (!rc) rc = make_bluestein(P, a);
  }
  if (rc) { delete P; return rc; }
  *out = P;
  return 0;
}

int hgp_plan_set_stream(hgp_plan* plan, void* hip_stream) {
  HGP_TRY(check_plan(plan));
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  if (s != plan->stream) {   // the plan's buffers may still be in use on the old stream
    HGP_TRY(use_device(plan));
    HIP_TRY(hipStreamSynchronize(plan->stream));
  }
  plan->stream = s;
  return 0;
}

int hgp_plan_set_column(hgp_plan* plan, const void* column, double jitter, double clamp_min, int64_t* n_clamped) {
  HGP_TRY(check_plan(plan));
  if (column == nullptr) return fail(HGP_E_ARG, "null column");
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, set_column_t, plan, column, jitter, clamp_min, n_clamped);
}

int hgp_toeplitz_apply(hgp_plan* plan, int op, const void* x, void* y, int64_t nrhs) {
  HGP_TRY(check_plan(plan));
  if (!plan->have_spec) return fail(HGP_E_STATE, "hgp_plan_set_column has not been called");
  if (op < HGP_OP_K || op > HGP_OP_R) return fail(HGP_E_ARG, "bad op");
  if (nrhs < 0 || (nrhs > 0 && (x == nullptr || y == nullptr))) return fail(HGP_E_ARG, "bad x/y/nrhs");
  if (x == y) return fail(HGP_E_ARG, "x and y must not alias");
  if (nrhs == 0) return 0;
  HGP_TRY(use_device(plan));
  hgp_plan* P = plan;
  hgp_plan::ApplyKey key;
  key.op = op; key.x = x; key.y = y; key.nrhs = nrhs; key.stream = P->stream;
  P->key_buffers(key);
  // a caller that is itself capturing (e.g. torch.cuda.graphs) records our launches directly
  hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(P->stream, &cst) != hipSuccess) { (void)hipGetLastError(); cst = hipStreamCaptureStatusActive; }
  if (!P->use_graphs || P->d < 2 || cst != hipStreamCaptureStatusNone)
    return DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr);
  if (P->graph_exec != nullptr && key == P->graph_key) {
    HIP_TRY(hipGraphLaunch(P->graph_exec, P->stream));
    return 0;
  }
  if (!(key == P->last_apply)) {
    // first call with these arguments: run it directly (workspaces are allocated here, so a
    // later capture never allocates); remember the workspaces it ended with
    HGP_TRY(DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr));
    P->key_buffers(key);
    P->last_apply = key;
    return 0;
  }
  // second identical call: capture the op's launches (all streams, fork/join events) once, on
  // the plan's capture stream (the graph is then launched on the caller's stream)
  P->drop_graph();
  if (P->cap_stream == nullptr) HIP_TRY(hipStreamCreateWithFlags(&P->cap_stream, hipStreamNonBlocking));
  hipGraph_t graph = nullptr;
  hipStream_t user = P->stream;
  if (hipStreamBeginCapture(P->cap_stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    (void)hipGetLastError();
    P->use_graphs = false;
    return DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr);
  }
  P->stream = P->cap_stream;
  const int rc = DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr);
  P->stream = user;
  const hipError_t ec = hipStreamEndCapture(P->cap_stream, &graph);
  if (rc != 0 || ec != hipSuccess || graph == nullptr) {
    if (graph) (void)hipGraphDestroy(graph);
    P->use_graphs = false;                      // fall back to direct launches for this plan
    (void)hipGetLastError();
    return rc != 0 ? rc : DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr);
  }
  hipGraphExec_t exec = nullptr;
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ei != hipSuccess) {
    P->use_graphs = false;
    (void)hipGetLastError();
    return DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr);
  }
  P->graph_exec = exec;
  P->graph_key = key;
  HIP_TRY(hipGraphLaunch(exec, P->stream));
  return 0;
}

int hgp_toeplitz_apply_pass(hgp_plan* plan, int op, const void* x, void* y, int64_t nrhs, int pass) {
  HGP_TRY(check_plan(plan));
  if (!plan->have_spec) return fail(HGP_E_STATE, "hgp_plan_set_column has not been called");
  if (op < HGP_OP_K || op > HGP_OP_R || pass < -1) return fail(HGP_E_ARG, "bad op/pass");
  if (nrhs <= 0 || x == nullptr || y == nullptr || x == y) return fail(HGP_E_ARG, "bad x/y/nrhs");
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, run_op, plan, op, x, y, nrhs, nullptr, nullptr, nullptr, pass);
}

int hgp_op_pass_count(const hgp_plan* plan) {
  if (plan == nullptr) return fail(HGP_E_ARG, "null plan");
  return plan->d == 1 ? 1 : (plan->d == 2 ? 3 : 5);
}

int hgp_pcg_begin(hgp_plan* plan, const void* b, void* x, int64_t nrhs, int use_precond, int layout) {
  HGP_TRY(check_plan(plan));
  if (!plan->have_spec) return fail(HGP_E_STATE, "hgp_plan_set_column has not been called");
  if (nrhs <= 0 || b == nullptr || x == nullptr) return fail(HGP_E_ARG, "bad b/x/nrhs");
  if (layout != HGP_LAYOUT_ROWS && layout != HGP_LAYOUT_COLS) return fail(HGP_E_ARG, "bad layout");
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, pcg_begin_t, plan, b, x, nrhs, use_precond ? 1 : 0, layout);
}

int hgp_pcg_step(hgp_plan* plan, double tol, int* converged) {
  HGP_TRY(check_plan(plan));
  if (!plan->cg_active) return fail(HGP_E_STATE, "hgp_pcg_begin has not been called");
  HGP_TRY(use_device(plan));
  HGP_TRY(DISPATCH(plan, pcg_step_t, plan, tol));
  HGP_TRY(DISPATCH(plan, pcg_finish_x, plan));
  if (converged) {
    int h = 0;
    HIP_TRY(hipMemcpyAsync(&h, plan->flags.ptr, sizeof(int), hipMemcpyDeviceToHost, plan->stream));
    HIP_TRY(hipStreamSynchronize(plan->stream));
    *converged = h != 0;
  }
  return 0;
}

int hgp_pcg_solve(hgp_plan* plan, const void* b, void* x, int64_t nrhs, int maxiter, double tol, int use_precond,
                  int layout, int* iters_done) {
  HGP_TRY(hgp_pcg_begin(plan, b, x, nrhs, use_precond, layout));
  // The break test runs on the device (every kernel after it is a no-op), so short solves
  // never synchronise.  Long ones (maxiter > 32, e.g. gram_solve's 2000) peek at the flag
  // every 16 iterations so that an early break also stops the host from queueing no-ops.
  const int chk = maxiter > 32 ? 16 : 0;
  for (int it = 0; it < maxiter; ++it) {
    HGP_TRY(DISPATCH(plan, pcg_step_t, plan, tol));
    if (chk && (it + 1) % chk == 0 && it + 1 < maxiter) {
      int h = 0;
      HIP_TRY(hipMemcpyAsync(&h, plan->flags.ptr, sizeof(int), hipMemcpyDeviceToHost, plan->stream));
      HIP_TRY(hipStreamSynchronize(plan->stream));
      if (h) break;
    }
  }
  HGP_TRY(DISPATCH(plan, pcg_finish_x, plan));
  if (iters_done) {
    int h[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(h, plan->flags.ptr, sizeof(h), hipMemcpyDeviceToHost, plan->stream));
    HIP_TRY(hipStreamSynchronize(plan->stream));
    *iters_done = h[1];
  }
  return 0;
}

int hgp_pcg_rnorm2(hgp_plan* plan, void* out) {
  HGP_TRY(check_plan(plan));
  if (!plan->cg_active) return fail(HGP_E_STATE, "hgp_pcg_begin has not been called");
  if (out == nullptr) return fail(HGP_E_ARG, "null out");
  HGP_TRY(use_device(plan));
  const size_t es = plan->dtype == HGP_F64 ? 8 : 4;
  const char* rnew = reinterpret_cast<const char*>(plan->scal.ptr) + 3 * plan->cg_nrhs * es;
  HIP_TRY(hipMemcpyAsync(out, rnew, plan->cg_nrhs * es, hipMemcpyDeviceToDevice, plan->stream));
  return 0;
}

int hgp_pcg_local_flag(hgp_plan* plan, double tol, int* flag) {
  HGP_TRY(check_plan(plan));
  if (!plan->cg_active) return fail(HGP_E_STATE, "hgp_pcg_begin has not been called");
  if (flag == nullptr) return fail(HGP_E_ARG, "null flag");
  HGP_TRY(use_device(plan));
  const void* rnew = reinterpret_cast<const char*>(plan->scal.ptr) + 3 * plan->cg_nrhs * plan->esz;
  if (plan->dtype == HGP_F64) cg_local_flag<double>(rnew, (int)plan->cg_nrhs, tol, flag, plan->stream);
  else cg_local_flag<float>(rnew, (int)plan->cg_nrhs, tol, flag, plan->stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hgp_pcg_iters(hgp_plan* plan, int* iters) {
  HGP_TRY(check_plan(plan));
  if (!plan->cg_active) return fail(HGP_E_STATE, "hgp_pcg_begin has not been called");
  if (iters == nullptr) return fail(HGP_E_ARG, "null iters");
  HGP_TRY(use_device(plan));
  int h[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(h, plan->flags.ptr, sizeof(h), hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  *iters = h[1];
  return 0;
}

int hgp_pcg_set_done(hgp_plan* plan, const int* flag) {
  HGP_TRY(check_plan(plan));
  if (!plan->cg_active) return fail(HGP_E_STATE, "hgp_pcg_begin has not been called");
  if (flag == nullptr) return fail(HGP_E_ARG, "null flag");
  HGP_TRY(use_device(plan));
  cg_set_done(reinterpret_cast<int*>(plan->flags.ptr), flag, plan->stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hgp_get_spectrum(hgp_plan* plan, int which, void* out) {
  HGP_TRY(check_plan(plan));
  if (!plan->have_spec) return fail(HGP_E_STATE, "hgp_plan_set_column has not been called");
  if (which < 0 || which > 2 || out == nullptr) return fail(HGP_E_ARG, "bad which/out");
  HGP_TRY(use_device(plan));
  GridDims g;
  g.d = plan->d;
  for (int a = 0; a < 3; ++a) { g.m[a] = plan->m[a]; g.n[a] = plan->n[a]; g.L[a] = plan->LK[a]; }
  const int sel = which == HGP_SPEC_D ? 0 : (which == HGP_SPEC_DI ? 1 : 2);   // Dm3 = [D | 1/D | sqrt D]
  const double* src = reinterpret_cast<const double*>(plan->Dm3.ptr) + sel * plan->M;
  if (plan->dtype == HGP_F64) expand_spec<double>(src, out, g, plan->stream);
  else expand_spec<float>(src, out, g, plan->stream);
  HIP_TRY(hipGetLastError());
  return 0;
}

int hgp_rowdot(int dtype, const void* a, const void* c, void* out, int64_t nrhs, int64_t M, void* hip_stream) {
  if (nrhs <= 0 || M <= 0) return 0;
  if (a == nullptr || c == nullptr || out == nullptr) return fail(HGP_E_ARG, "null pointer");
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  hipStream_t s = reinterpret_cast<hipStream_t>(hip_stream);
  const int np = update_np(M);
  const size_t es = dtype == HGP_F64 ? 8 : 4;
  // partial sums in a per-thread, per-device scratch that persists across calls: a call on
  // another stream first waits for the previous user's event, growth waits for it on the host
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  // (heap-held and never destroyed: no hipFree runs during process teardown)
  static thread_local std::vector<RowdotScratch>* pool = new std::vector<RowdotScratch>();
  RowdotScratch* sc = nullptr;
  for (auto& e : *pool)
    if (e.device == dev) sc = &e;
  if (sc == nullptr) {
    pool->emplace_back();
    sc = &pool->back();
    sc->device = dev;
    HIP_TRY(hipEventCreateWithFlags(&sc->ev, hipEventDisableTiming));
  }
  const size_t need = (size_t)(nrhs * np) * es;
  if (sc->used && need > sc->buf.bytes) HIP_TRY(hipEventSynchronize(sc->ev));
  HGP_TRY(sc->buf.ensure(need));
  if (sc->used && sc->last != s) HIP_TRY(hipStreamWaitEvent(s, sc->ev, 0));
  void* part = sc->buf.ptr;
  if (dtype == HGP_F64) { rowdot_part<double>(a, c, part, nrhs, M, np, s); reduce_rows<double>(part, np, (int)nrhs, out, s); }
  else { rowdot_part<float>(a, c, part, nrhs, M, np, s); reduce_rows<float>(part, np, (int)nrhs, out, s); }
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(sc->ev, s));
  sc->last = s;
  sc->used = true;
  return 0;
}

int hgp_kuf_grid(int dtype, int kind, int ndim, const int64_t* m, const void* const* grids, const void* x,
                 int64_t nobs, double sig2, double ell, void* out, void* hip_stream) {
  if (ndim < 1 || ndim > 3 || m == nullptr || grids == nullptr) return fail(HGP_E_ARG, "ndim must be 1..3, m/grids non-null");
  if (kind < HGP_KERN_SQEXP || kind > HGP_KERN_MATERN52) return fail(HGP_E_ARG, "bad kernel kind");
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (nobs == 0) return 0;
  if (nobs < 0 || x == nullptr || out == nullptr) return fail(HGP_E_ARG, "bad x/out/nobs");
  for (int a = 0; a < ndim; ++a)
    if (m[a] < 1 || grids[a] == nullptr) return fail(HGP_E_ARG, "grid sizes must be >= 1 with non-null grids");
  hipError_t e = kuf_grid(dtype, kind, ndim, m, grids, x, nobs, sig2, ell, out, reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_kuf_grid: ") + hipGetErrorString(e));
  return 0;
}

static int check_grid_args(int dtype, int ndim, const int64_t* m, const void* const* grids, const void* x,
                           int64_t nobs, const void* out) {
  if (ndim < 1 || ndim > 3 || m == nullptr || grids == nullptr) return fail(HGP_E_ARG, "ndim must be 1..3, m/grids non-null");
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (nobs < 0 || (nobs > 0 && (x == nullptr || out == nullptr))) return fail(HGP_E_ARG, "bad x/out/nobs");
  for (int a = 0; a < ndim; ++a)
    if (m[a] < 1 || grids[a] == nullptr) return fail(HGP_E_ARG, "grid sizes must be >= 1 with non-null grids");
  return 0;
}

int hgp_kuf_semi_mc(int dtype, int kind, double kparam, int ndim, const int64_t* m, const void* const* grids,
                    const void* x, int64_t nobs, double sig2, double ell, int npts, const void* u, void* out,
                    void* hip_stream) {
  HGP_TRY(check_grid_args(dtype, ndim, m, grids, x, nobs, out));
  if (kind < HGP_KERN_SQEXP || kind > HGP_KERN_GNEITING) return fail(HGP_E_ARG, "bad kernel kind");
  if (npts < 1 || npts > 1024) return fail(HGP_E_ARG, "npts must be in [1, 1024]");
  if (u == nullptr) return fail(HGP_E_ARG, "u (the device offset draw) is null");
  if (nobs == 0) return 0;
  hipError_t e = kuf_semi(dtype, kind, kparam, ndim, m, grids, x, nobs, sig2, ell, npts, u, out,
                          reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_kuf_semi_mc: ") + hipGetErrorString(e));
  return 0;
}

int hgp_kuf_semi_sqexp(int dtype, int ndim, const int64_t* m, const void* const* grids, const void* x, int64_t nobs,
                       double sig2, double ell, void* out, void* hip_stream) {
  HGP_TRY(check_grid_args(dtype, ndim, m, grids, x, nobs, out));
  if (nobs == 0) return 0;
  hipError_t e = kuf_semi(dtype, HGP_KERN_SQEXP, 1.0, ndim, m, grids, x, nobs, sig2, ell, 0, nullptr, out,
                          reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_kuf_semi_sqexp: ") + hipGetErrorString(e));
  return 0;
}

int hgp_knn_doubly_diag(int dtype, int ndim, const void* x, int64_t nobs, double sig2, double ell, const void* table,
                        int N, void* out, void* hip_stream) {
  if (ndim < 1 || ndim > 3) return fail(HGP_E_ARG, "ndim must be 1..3");
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (N < 2 || table == nullptr) return fail(HGP_E_ARG, "table needs N >= 2 entries");
  if (nobs < 0 || (nobs > 0 && (x == nullptr || out == nullptr))) return fail(HGP_E_ARG, "bad x/out/nobs");
  if (nobs == 0) return 0;
  hipError_t e = doubly_diag(dtype, ndim, x, nobs, sig2, ell, table, N, out, reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_knn_doubly_diag: ") + hipGetErrorString(e));
  return 0;
}

int hgp_meanfield_stats(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                        const void* y, const void* ivar, const void* Knn_diag, const void* log_sd, void* an, void* lam,
                        void* dm, void* hip_stream) {
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (nrhs < 0 || Mp <= 0) return fail(HGP_E_ARG, "nrhs >= 0 and Mp > 0 required");
  if (kn == nullptr || qm == nullptr || qS == nullptr || lam == nullptr || dm == nullptr ||
      (nrhs > 0 && (y == nullptr || ivar == nullptr || Knn_diag == nullptr || log_sd == nullptr || an == nullptr)))
    return fail(HGP_E_ARG, "null pointer");
  hipError_t e = meanfield_stats(dtype, kn, nrhs, Mp, qm, qS, y, ivar, Knn_diag, log_sd, an, lam, dm,
                                 reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_meanfield_stats: ") + hipGetErrorString(e));
  return 0;
}

int hgp_meanfield_rowdots(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* qm, const void* qS,
                          void* out3, void* hip_stream) {
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (nrhs < 0 || Mp < 0) return fail(HGP_E_ARG, "nrhs >= 0 and Mp >= 0 required");
  if (nrhs > 0 && (out3 == nullptr || (Mp > 0 && (kn == nullptr || qm == nullptr || qS == nullptr))))
    return fail(HGP_E_ARG, "null pointer");
  hipError_t e = meanfield_rowdots(dtype, kn, nrhs, Mp, qm, qS, out3, reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_meanfield_rowdots: ") + hipGetErrorString(e));
  return 0;
}

int hgp_meanfield_cols(int dtype, const void* kn, int64_t nrhs, int64_t Mp, const void* ivar, const void* bdiff,
                       void* lam, void* dm, void* hip_stream) {
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (nrhs < 0 || Mp < 0) return fail(HGP_E_ARG, "nrhs >= 0 and Mp >= 0 required");
  if (Mp > 0 && (lam == nullptr || dm == nullptr || (nrhs > 0 && (kn == nullptr || ivar == nullptr || bdiff == nullptr))))
    return fail(HGP_E_ARG, "null pointer");
  hipError_t e = meanfield_cols(dtype, kn, nrhs, Mp, ivar, bdiff, lam, dm, reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_meanfield_cols: ") + hipGetErrorString(e));
  return 0;
}

int hgp_block_stats(int dtype, int ndim, const int64_t* dims, const int64_t* blocks, const void* kn, int64_t nrhs,
                    const void* ivar, const void* S, void* gram, void* knSkn, void* trSG, void* hip_stream) {
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "dtype must be HGP_F32 or HGP_F64");
  if (dims == nullptr || blocks == nullptr) return fail(HGP_E_ARG, "null dims/blocks");
  if (nrhs < 0 || nrhs > (int64_t)1 << 30) return fail(HGP_E_ARG, "nrhs out of range");
  BlockGeom g;
  const char* why = nullptr;
  if (block_geom(ndim, dims, blocks, &g, &why) != 0) return fail(HGP_E_UNSUPPORTED, std::string("hgp_block_stats: ") + why);
  if (gram == nullptr && knSkn == nullptr && trSG == nullptr) return 0;
  if (trSG != nullptr && gram == nullptr) return fail(HGP_E_ARG, "trSG needs the gram output");
  if (nrhs > 0 && kn == nullptr) return fail(HGP_E_ARG, "null kn");
  if (gram != nullptr && nrhs > 0 && ivar == nullptr) return fail(HGP_E_ARG, "null ivar");
  if ((knSkn != nullptr || trSG != nullptr) && S == nullptr) return fail(HGP_E_ARG, "null S");
  hipError_t e = block_stats(dtype, g, kn, nrhs, ivar, S, gram, knSkn, trSG, reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_block_stats: ") + hipGetErrorString(e));
  return 0;
}

int hgp_sym_toeplitz_dqf(int dtype, const void* left, const void* right, int64_t nvec, int64_t n, void* out,
                         void* hip_stream) {
  if (dtype != HGP_F32 && dtype != HGP_F64) return fail(HGP_E_ARG, "bad dtype");
  if (nvec < 0 || n <= 0) return fail(HGP_E_ARG, "bad nvec/n");
  if (out == nullptr || (nvec > 0 && (left == nullptr || right == nullptr))) return fail(HGP_E_ARG, "null pointer");
  hipError_t e = sym_toeplitz_dqf(dtype, left, right, nvec, n, out, reinterpret_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(HGP_E_HIP, std::string("hgp_sym_toeplitz_dqf: ") + hipGetErrorString(e));
  return 0;
}

// F = FFT_L(conj(sum_b conj(V_b) H_b)) on the L-grid (L = L_K or L_R, fp64): Re F[t mod L] / prod L
// = sum_b sum_j v_b[j] h_b[j + t] (hgp_grad.hip).  v rows on the m-grid (stride M); h rows on the
// m-grid (zero-padded) or, h_periodic, on the n-grid (stride M').  Scratch: three L-grids.
int xcorr_grid(hgp_plan* P, int useR, const void* v, const void* h, int h_periodic, int64_t nb, DevBuf* buf,
               double2** F, GridDims* gout) {
  hipStream_t s = P->stream;
  const int64_t* L = useR ? P->LR : P->LK;
  const DevBuf* tw = useR ? P->tw64R : P->tw64K;
  const int64_t prodL = useR ? P->prodLR : P->prodLK;
  GridDims gd;
  gd.d = P->d;
  for (int a = 0; a < 3; ++a) { gd.m[a] = P->m[a]; gd.n[a] = P->n[a]; gd.L[a] = L[a]; }
  // (one spare double2 after S holds the packing maxima of the current RHS)
  for (int i = 0; i < 3; ++i) HGP_TRY(buf[i].ensure((size_t)(prodL + (i == 2 ? 1 : 0)) * sizeof(double2)));
  double2* z = reinterpret_cast<double2*>(buf[0].ptr);
  double2* w = reinterpret_cast<double2*>(buf[1].ptr);
  double2* S = reinterpret_cast<double2*>(buf[2].ptr);
  unsigned long long* mx = reinterpret_cast<unsigned long long*>(S + prodL);
  const size_t es = P->esz;
  const int64_t hs = h_periodic ? P->Mp : P->M;
  for (int64_t b = 0; b < nb; ++b) {
    pack_pair(P->dtype, static_cast<const char*>(v) + (size_t)(b * P->M) * es,
              static_cast<const char*>(h) + (size_t)(b * hs) * es, h_periodic, gd, prodL, z, mx, P->M, hs, s);
    double2* Z = nullptr;
    HGP_TRY(fwd_grid_f64(P, L, tw, z, w, &Z));
    xspec_acc(Z, S, gd, prodL, b == 0 ? 1 : 0, mx, s);
  }
  if (nb == 0) HIP_TRY(hipMemsetAsync(S, 0, (size_t)prodL * sizeof(double2), s));
  conj_inplace(S, prodL, s);
  HGP_TRY(fwd_grid_f64(P, L, tw, S, z, F));
  HIP_TRY(hipGetLastError());
  *gout = gd;
  return 0;
}

// d/dcolumn <g, op x> through the operator's spectrum S(D) (toeplitz_tensor.py:20-31, ops :70-125).
// With A = DCT-I on the m-grid (A[f][x] = mu(x) cos(2 pi f x / n) per axis, dct_axis), D = A column
// and the operator's generator c = A S(D) / N on the n-grid:
//   gs = fold(X) (X = dL/dc on the n-grid, hgp_grad.hip), dL/dS = A^T gs / N,
//   dL/dD = dL/dS * S'(D) * [D > cmin], dL/dcolumn = A^T dL/dD,  A^T y = mu (A (y / mu)).
int hgp_plan_column_grad(hgp_plan* plan, int op, const void* x, const void* g, int64_t nrhs, void* column_grad) {
  HGP_TRY(check_plan(plan));
  if (!plan->have_spec) return fail(HGP_E_STATE, "hgp_plan_set_column has not been called");
  if (op < HGP_OP_K || op > HGP_OP_R) return fail(HGP_E_ARG, "bad op");
  if (nrhs < 0 || column_grad == nullptr || (nrhs > 0 && (x == nullptr || g == nullptr)))
    return fail(HGP_E_ARG, "bad nrhs or null pointer");
  if (plan->d < 1) return fail(HGP_E_UNSUPPORTED, "a grid with a single point has no column gradient");
  HGP_TRY(use_device(plan));
  hgp_plan* P = plan;
  hipStream_t s = P->stream;
  const int64_t M = P->M, Mp = P->Mp;
  GridDims gd;
  gd.d = P->d;
  for (int a = 0; a < 3; ++a) { gd.m[a] = P->m[a]; gd.n[a] = P->n[a]; gd.L[a] = P->LK[a]; }
  DevBuf X, y1, y2, big[3];   // freed on return (after the stream sync below)
  HGP_TRY(X.ensure((size_t)Mp * sizeof(double)));
  HGP_TRY(y1.ensure((size_t)M * sizeof(double)));
  HGP_TRY(y2.ensure((size_t)M * sizeof(double)));
  double* Xp = reinterpret_cast<double*>(X.ptr);
  double* a = reinterpret_cast<double*>(y1.ptr);
  double* b = reinterpret_cast<double*>(y2.ptr);
  {
    // <g, op x> = sum_b sum_{j in m-grid} v_b[j] sum_w c[w] h_b[(j + w) mod n] with (v, h) =
    // (x, g) for R^T (g on the n-grid), (g, x) for R (x on the n-grid), (x, g) for K / C^-1
    // (g on the m-grid, zero elsewhere: the crop); X[w] = dL/dc[w] by one cross spectrum
    const void* vv = op == HGP_OP_R ? g : x;
    const void* hh = op == HGP_OP_R ? x : g;
    const int periodic = (op == HGP_OP_R || op == HGP_OP_RT) ? 1 : 0;
    double2* F = nullptr;
    GridDims gl;
    HGP_TRY(xcorr_grid(P, periodic, vv, hh, periodic, nrhs, big, &F, &gl));
    gather_n(F, gl, periodic, Mp, 1.0 / (double)(periodic ? P->prodLR : P->prodLK), Xp, s);
  }
  fold_div_mu(Xp, M, gd, a, s);
  for (int ax = 0; ax < P->d; ++ax) {
    HGP_TRY(dct_axis(P, ax, a, b, 1, 1.0 / (double)P->n[ax]));
    std::swap(a, b);
  }
  const int kind = op == HGP_OP_K ? 0 : (op == HGP_OP_CINV ? 1 : 2);
  spec_bwd(a, reinterpret_cast<const double*>(P->Dm3.ptr), M, kind, P->clamp_min, s);
  for (int ax = 0; ax < P->d; ++ax) {
    HGP_TRY(dct_axis(P, ax, a, b, 1, 1.0));
    std::swap(a, b);
  }
  mul_mu_out(P->dtype, a, M, gd, column_grad, s);
  HIP_TRY(hipGetLastError());
  // the scratch is freed on return: finish its users first
  HIP_TRY(hipStreamSynchronize(s));
  return 0;
}

int hgp_plan_dqf(hgp_plan* plan, const void* left, const void* right, int64_t nvec, void* out) {
  HGP_TRY(check_plan(plan));
  if (nvec < 0 || out == nullptr || (nvec > 0 && (left == nullptr || right == nullptr)))
    return fail(HGP_E_ARG, "bad nvec or null pointer");
  if (plan->d < 1) return fail(HGP_E_UNSUPPORTED, "a grid with a single point");
  HGP_TRY(use_device(plan));
  DevBuf big[3];
  double2* F = nullptr;
  GridDims gl;
  HGP_TRY(xcorr_grid(plan, 0, left, right, 0, nvec, big, &F, &gl));
  gather_flat(plan->dtype, F, gl, plan->M, 1.0 / (double)plan->prodLK, out, plan->stream);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(plan->stream));
  return 0;
}

int hgp_slab_info(const hgp_plan* plan, int op, int64_t* ngroups, int64_t* inner) {
  HGP_TRY(check_plan(plan));
  if (op < HGP_OP_K || op > HGP_OP_R) return fail(HGP_E_ARG, "bad op");
  if (plan->d < 2) return fail(HGP_E_UNSUPPORTED, "slab sharding needs a 2-D or 3-D grid");
  const SlabGeom g = slab_geom(plan, op);
  if (ngroups) *ngroups = g.NG;
  if (inner) *inner = g.inner;
  return 0;
}

int hgp_slab_pass_ex(hgp_plan* plan, int op, int stage, const void* in, void* out, int64_t nrhs, int64_t nrows,
                     int64_t g0, int64_t ng, const void* dotv, void* dot_out, const int* done) {
  HGP_TRY(check_plan(plan));
  if (!plan->have_spec) return fail(HGP_E_STATE, "hgp_plan_set_column has not been called");
  if (op < HGP_OP_K || op > HGP_OP_R) return fail(HGP_E_ARG, "bad op");
  if (plan->d < 2) return fail(HGP_E_UNSUPPORTED, "slab sharding needs a 2-D or 3-D grid");
  if (stage < HGP_SLAB_FWD || stage > HGP_SLAB_CONV_A2A) return fail(HGP_E_ARG, "bad slab stage");
  if (nrhs < 0 || (nrhs > 0 && (in == nullptr || out == nullptr))) return fail(HGP_E_ARG, "bad in/out/nrhs");
  if (stage != HGP_SLAB_CONV && in == out) return fail(HGP_E_ARG, "in and out must not alias (row stages)");
  if (dotv != nullptr && (stage != HGP_SLAB_INV || dot_out == nullptr))
    return fail(HGP_E_ARG, "a fused dot (dotv, dot_out) is an HGP_SLAB_INV option and needs both pointers");
  if (nrhs == 0) return 0;
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, slab_pass_t, plan, op, stage, in, out, nrhs, nrows, g0, ng, dotv, dot_out, done);
}

int hgp_slab_pass(hgp_plan* plan, int op, int stage, const void* in, void* out, int64_t nrhs, int64_t nrows,
                  int64_t g0, int64_t ng) {
  return hgp_slab_pass_ex(plan, op, stage, in, out, nrhs, nrows, g0, ng, nullptr, nullptr, nullptr);
}

}  // extern "C"

// ---- slab-sharded PCG scalars (cg.py:63-78 on all-reduced per-RHS dots) --------------------
template <typename T>
int slab_cg_xr_t(hgp_plan* P, void* x, void* r, const void* p, const void* Ap, const void* rs, const void* pAp,
                 void* rr, int64_t nrhs, int64_t M, const int* done) {
  hipStream_t st = P->stream;
  if (M == 0) {             // a rank without rows: its share of r.r is 0
    HIP_TRY(hipMemsetAsync(rr, 0, (size_t)nrhs * sizeof(T), st));
    return 0;
  }
  const int np = update_np(M);
  HGP_TRY(P->slab_coef.ensure((size_t)nrhs * sizeof(T)));
  HGP_TRY(P->slab_part.ensure((size_t)(nrhs * np) * sizeof(T)));
  cg_alpha<T>(pAp, 1, (int)nrhs, rs, P->slab_coef.ptr, done, st);                 // alpha = rs / p.Ap
  cg_update_xr<T>(x, r, p, Ap, P->slab_coef.ptr, P->slab_part.ptr, nrhs, M, done, st);
  reduce_rows<T>(P->slab_part.ptr, np, (int)nrhs, rr, st);                         // local r.r
  return 0;
}

template <typename T>
int slab_cg_check_t(hgp_plan* P, const void* rr, int64_t nrhs, double tol, int* done, int* iters) {
  // rr are the all-reduced r.r: done = the iteration when every sqrt(r.r) < tol (cg.py:69-71);
  // k_cg_check writes rnew = the reduced sums again, so it gets a scratch copy
  HGP_TRY(P->slab_coef.ensure((size_t)nrhs * sizeof(T)));
  cg_check<T>(rr, 1, (int)nrhs, tol, P->slab_coef.ptr, done, iters, P->stream);
  return 0;
}

template <typename T>
int slab_cg_p_t(hgp_plan* P, void* p, const void* z, void* rs, const void* zr, int64_t nrhs, int64_t M,
                const int* done) {
  HGP_TRY(P->slab_coef.ensure((size_t)nrhs * sizeof(T)));
  cg_beta<T>(zr, 1, (int)nrhs, rs, P->slab_coef.ptr, done, P->stream);           // beta = zr / rs; rs = zr
  if (M > 0) cg_update_p<T>(p, z, P->slab_coef.ptr, nrhs, M, done, P->stream);    // p = z + beta p
  return 0;
}

extern "C" {

static int slab_cg_args(const hgp_plan* plan, int64_t nrhs, int64_t M, const int* done) {
  HGP_TRY(check_plan(plan));
  if (nrhs < 1 || M < 0 || done == nullptr) return fail(HGP_E_ARG, "bad nrhs / M / done");
  return 0;
}

int hgp_slab_cg_xr(hgp_plan* plan, void* x, void* r, const void* p, const void* Ap, const void* rs, const void* pAp,
                   void* rr, int64_t nrhs, int64_t M, const int* done) {
  HGP_TRY(slab_cg_args(plan, nrhs, M, done));
  if (rs == nullptr || pAp == nullptr || rr == nullptr || (M > 0 && (!x || !r || !p || !Ap)))
    return fail(HGP_E_ARG, "null vector / scalar");
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, slab_cg_xr_t, plan, x, r, p, Ap, rs, pAp, rr, nrhs, M, done);
}

int hgp_slab_cg_check(hgp_plan* plan, const void* rr, int64_t nrhs, double tol, int* done, int* iters) {
  HGP_TRY(slab_cg_args(plan, nrhs, 0, done));
  if (rr == nullptr || iters == nullptr) return fail(HGP_E_ARG, "null rr / iters");
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, slab_cg_check_t, plan, rr, nrhs, tol, done, iters);
}

int hgp_slab_cg_p(hgp_plan* plan, void* p, const void* z, void* rs, const void* zr, int64_t nrhs, int64_t M,
                  const int* done) {
  HGP_TRY(slab_cg_args(plan, nrhs, M, done));
  if (rs == nullptr || zr == nullptr || (M > 0 && (!p || !z))) return fail(HGP_E_ARG, "null vector / scalar");
  HGP_TRY(use_device(plan));
  return DISPATCH(plan, slab_cg_p_t, plan, p, z, rs, zr, nrhs, M, done);
}

int hgp_plan_info(const hgp_plan* plan, int64_t* M, int64_t* Mprime, int64_t* L_K, int64_t* L_R) {
  HGP_TRY(check_plan(plan));
  if (M) *M = plan->M;
  if (Mprime) *Mprime = plan->Mp;
  for (int a = 0; a < 3; ++a) {
    if (L_K) L_K[a] = a < plan->d ? plan->LK[a] : 1;
    if (L_R) L_R[a] = a < plan->d ? plan->LR[a] : 1;
  }
  return 0;
}

int64_t plan_scratch_bytes(const hgp_plan* P) {
  const DevBuf* bufs[] = {&P->ws1, &P->ws2, &P->set1, &P->set2, &P->setM1, &P->setM2, &P->setC, &P->r, &P->z,
                          &P->p, &P->Ap, &P->part_op, &P->part_u, &P->part_f, &P->scal, &P->bT, &P->xT,
                          &P->gridA, &P->gridB,    // the full-grid R / R^T buffers (grid_r plans)
                          &P->slab_part, &P->slab_coef};
  int64_t b = 0;
  for (const DevBuf* d : bufs) b += (int64_t)d->bytes;
  return b;
}

int hgp_plan_mem(const hgp_plan* plan, int64_t* scratch_bytes, int64_t* table_bytes) {
  HGP_TRY(check_plan(plan));
  if (scratch_bytes) *scratch_bytes = plan_scratch_bytes(plan);
  if (table_bytes) {
    int64_t b = 0;
    for (int a = 0; a < 3; ++a)
      b += (int64_t)(plan->twK[a].bytes + plan->twR[a].bytes + plan->tw64K[a].bytes + plan->tw64R[a].bytes +
                     plan->bsPre[a].bytes + plan->bsPost[a].bytes + plan->bsFilt[a].bytes);
    b += (int64_t)(plan->specK.bytes + plan->specI.bytes + plan->specR.bytes + plan->specRg.bytes + plan->specKg.bytes +
                   plan->Dm3.bytes);
    *table_bytes = b;
  }
  return 0;
}

int hgp_plan_trim(hgp_plan* plan) {
  HGP_TRY(check_plan(plan));
  if (plan->cg_active) plan->cg_active = false;   // the CG state goes with its buffers
  HGP_TRY(use_device(plan));
  HIP_TRY(hipStreamSynchronize(plan->stream));     // no kernel may still use them
  for (int i = 0; i < 3; ++i)
    if (plan->side[i]) HIP_TRY(hipStreamSynchronize(plan->side[i]));
  DevBuf* bufs[] = {&plan->ws1, &plan->ws2, &plan->set1, &plan->set2, &plan->setM1, &plan->setM2, &plan->setC,
                    &plan->r, &plan->z, &plan->p, &plan->Ap, &plan->part_op, &plan->part_u, &plan->part_f,
                    &plan->scal, &plan->bT, &plan->xT, &plan->gridA, &plan->gridB, &plan->slab_part,
                    &plan->slab_coef};
  for (DevBuf* b : bufs) b->release();
  plan->drop_graph();                               // its kernels addressed the freed workspaces
  plan->last_apply = hgp_plan::ApplyKey();
  return 0;
}

int hgp_plan_destroy(hgp_plan* plan) {
  if (plan == nullptr) return 0;
  (void)hipSetDevice(plan->device);
  (void)hipStreamSynchronize(plan->stream);
  delete plan;
  return 0;
}

}  // extern "C"
