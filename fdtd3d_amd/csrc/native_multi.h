// native_multi.h -- --parallel-grid decompositions (x / y / z rank grids) driven from one process.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "capi.h"
#include "host_native.h"
#include "settings_native.h"
#include "native_api.h"
#include "native_setup.h"
#include "native_ckpt.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
namespace {

// ------------------------------------------------------------ multi-GPU
// --parallel-grid: the 3D grid split over a Px x Py x Pz rank grid
// (--topology-sizex/y/z; none given: one x slab per visible GPU), every rank
// driven by this one process (rank r on device r % devices).  Every T steps
// each rank runs the temporally blocked kernel over its owned cells, reading
// T-deep ghosts (the pass's dependency cone); then it packs, for each of its
// up to 26 face / edge / corner neighbours, the owned T-deep box that
// neighbour holds as ghosts (one kernel, six components); at the next pass
// each rank pulls its neighbours' packed boxes (xGMI peer copies between
// devices) and unpacks them into its ghosts on a side stream while its main
// stream runs the interior (cells that need no fresh ghost), then the
// T-thick shells -- the direct 26-neighbour exchange of parallel/halo.py
// overlapped as models/blocking.py _tb_step does, point-to-point only, the
// shape of the node's xGMI links.  Plain Yee
// media (vacuum / dielectric sphere) with the point source; the reference's
// MPI grid: Source/Grid/ParallelGrid.cpp:1600-1823 (exchange), :2161-2194.
//
// Physics (CPML absorbing layers, TF/SF plane waves, point source, vacuum or
// the dielectric sphere): every rank steps its owned cells with the split
// half-step kernels of the single-GPU stepped path (the folded 4-cell-lane
// CPML kernels, the TF/SF correction tables, the incident line), and the
// updated kind's three components go to the face neighbours after every half
// step -- one-cell ghosts in x / y, 4-cell ghosts in z (whole lanes), the
// reference's buffer-size-1 exchange (ParallelGrid.cpp:1600-1823 after each
// of performExSteps / performHxSteps, Scheme3D.cpp:1900-2942).  The CPML
// profiles, psi slabs and TF/SF targets are built per rank from the global
// positions (native_setup.h setup_cpml / setup_tfsf with the rank's origin),
// so no psi ever needs a ghost: ghosts are read, never updated.
template <typename T>
struct XRank {
  int dev = 0;
  hipStream_t st = nullptr, side = nullptr;  // passes / ghost pulls
  hipEvent_t done = nullptr, copied = nullptr;
  std::vector<std::array<int, 6>> outs;      // output boxes of a pass: interior, then the shells
  int crd[3] = {0, 0, 0};
  int lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};  // owned global range
  int g0[3] = {0, 0, 0}, n[3] = {0, 0, 0};   // allocated box (ghosts included): global origin, extent
  Dev<T> F[6], G[6], C[6];
  int boxes[36];
  // per direction d (0..26, 13 = self): the owned box sent to the neighbour
  // at d and the ghost box received from it (local indices), its buffers
  int nb[27];
  int sbox[27][6], rbox[27][6];
  Dev<T> sbuf[27], rbuf[27];
  // physics: the owned part of every component's update range (local
  // indices), the rank's CPML tables, TF/SF tables and incident line, the
  // point source's local offset (-1: not owned)
  int own36[36];
  std::unique_ptr<NativeCpml<T>> cp;
  std::unique_ptr<NativeTfsf<T>> tf;
  // UPML / Drude: the rank's chain tables and region-local D levels, its part
  // of the global chain and plain regions (local indices)
  std::unique_ptr<native_phys::Upml<T>> up;
  // 2D: the CPML slabs / UPML strips tables and the half-step helper
  std::unique_ptr<Pml2d<T>> p2;
  std::unique_ptr<Lowdim2d<T>> ld;
  std::vector<IBox> chain_regs, plain_regs;
  std::vector<bool> chain_disp;
  long long src_off = -1;
  // amplitude mode: running maxima ([x][6][y][z]), changed counts of a
  // check period, the amplitude boxes (local), the z-line cells it owns,
  // the near-convergence snapshot
  Dev<T> AMP;
  Dev<unsigned> CNT;
  Dev<long long> LINE;
  int line_n = 0;
  int ab[36];
  Dev<char> SNAP;
  size_t cells() const { return (size_t)n[0] * n[1] * n[2]; }
};

template <typename T>
class MultiRun {
 public:
  explicit MultiRun(const fdtd::Settings& s_) : s(s_) {}
  ~MultiRun() { release(); }
  int main();

 private:
  const fdtd::Settings& s;
  fdtd::Int3 N;
  int dim = 3;
  std::string scheme = "3d";
  std::vector<int> active = {0, 1, 2};
  bool present[6] = {true, true, true, true, true, true};
  int src_comp = 2;
  double dt = 0, freq = 0, cb = 0, db = 0;
  bool percell = false;
  bool phys = false, cpml = false, upml = false, tfsf = false, point_src = true, ntff = false;
  bool amp = false, amp_on = false, amp_line = false;  // amplitude mode; its phase; the global z line exists
  int amp_taken = 0, amp_stable = -1;
  Dev<T> NG[6];  // NTFF: the whole grid assembled on the first rank's device
  double ckpt_ms = 0.0;
  int ndev = 0, P = 1, TB = 1;
  int Pd[3] = {1, 1, 1};
  int gd[3] = {1, 1, 1};  // ghost depth per axis
  fdtd::Int3 sp;
  std::vector<XRank<T>> R;
  bool first = true;

  double src_val(int t) const {
    if (s.sourceType == "gaussian") return std::exp(-std::pow((t - s.gaussianDelay) / s.gaussianWidth, 2));
    return std::sin(dt * t * 2 * kPi * freq);
  }
  int rank_of(const int* c) const { return (c[0] * Pd[1] + c[1]) * Pd[2] + c[2]; }
  int plan_ranks();
  void setup_rank(int r);
  void enable_peers();
  void plan_outputs();
  void pull_ghosts();
  void rank_pass(XRank<T>& q, int t, int k);
  void pass(int t, int k);
  bool setup_physics(int r);
  void setup_chain(XRank<T>& q);
  static void clip36(const int* b36, const IBox& r, int* out);
  void phys_half(XRank<T>& q, int kind, double sv);
  void exchange(int kind);
  void phys_step(int t);
  void setup_amp(XRank<T>& q);
  std::vector<std::pair<void*, size_t>> rank_state(XRank<T>& q);
  int amp_run(int t);
  void advance(int t0, int n);
  void run_steps(int t0, int n);
  void run_ckpt(int t, int n);
  void gather(int c, std::vector<T>& host);
  void scatter(int c, const std::vector<T>& host);
  void ntff_report(int t);
  void sync_all();
  void report(double sec, int t_end, int steps, int warm) const;
  bool save_results(int steps);
  void release();
};

// the rank grid (--topology-sizex/y/z, else one x slab per GPU), the steps
// per pass and every rank's owned / allocated box; 2 when the grid does not
// split that way
template <typename T>
int MultiRun<T>::plan_ranks() {
  dim = s.dimension;
  scheme = dim == 3 ? "3d" : (dim == 2 ? s.mode2D : "1d");
  N = {s.sizeX, dim >= 2 ? s.sizeY : 1, dim == 3 ? s.sizeZ : 1};
  if (dim == 1) {
    // Ez / Hy on x slabs
    active = {0};
    for (int c = 0; c < 6; ++c) present[c] = c == 2 || c == 4;
  }
  if (dim == 2) {
    // TMz (Ez Hx Hy) / TEz (Ex Ey Hz) on an x / y rank grid
    active = {0, 1};
    for (int c = 0; c < 6; ++c) present[c] = false;
    if (scheme == "tmz") present[2] = present[3] = present[4] = true;
    else present[0] = present[1] = present[5] = true;
    src_comp = scheme == "tmz" ? 2 : 5;
  }
  const double dx = s.gridStep;
  dt = dx * s.courantNum / kC;
  freq = kC / s.sourceWaveLength;
  cb = dt / (kEps0 * dx);
  db = dt / (kMu0 * dx);
  percell = s.scene != "vacuum" && s.scene != "drude-sphere";  // (a Drude sphere's eps_inf is 1)
  HIP_OK(hipGetDeviceCount(&ndev));
  Pd[0] = std::max(1, s.topologySizeX);
  Pd[1] = std::max(1, s.topologySizeY);
  Pd[1] = dim >= 2 ? Pd[1] : 1;
  Pd[2] = dim == 3 ? std::max(1, s.topologySizeZ) : 1;
  if (Pd[0] * Pd[1] * Pd[2] == 1) Pd[0] = ndev;
  P = Pd[0] * Pd[1] * Pd[2];
  upml = (s.doUsePML && s.pmlType == "upml") || s.doUseMetamaterials;  // the D/B chain
  cpml = s.doUsePML && !upml;
  tfsf = s.doUseTFSF;
  amp = s.doUseAmplitudeMode;
  phys = cpml || upml || tfsf || amp || dim < 3;  // (1D / 2D: the split half steps always)
  ntff = s.doUseNTFF && dim == 3;
  point_src = !tfsf || s.doUsePointSource;
  const int T_max = sizeof(T) == 4 ? fdtd_tb_max_steps() : fdtd_tb64_max_steps();
  TB = phys ? 1 : std::max(1, std::min(T_max, s.timeBlock <= 0 ? (sizeof(T) == 4 ? 5 : 4) : s.timeBlock));
  for (int a = 0; a < 3; ++a) gd[a] = TB;
  if (phys) gd[2] = Pd[2] > 1 ? 4 : 1;  // z ghosts of whole 4-cell lanes
  for (int a = 0; a < 3; ++a)
    if (N[a] / Pd[a] < gd[a]) {
      std::fprintf(stderr, "fdtd3d (native): %d cells along axis %d over %d ranks leave fewer than %d per rank\n",
                   N[a], a, Pd[a], gd[a]);
      return 2;
    }
  R.resize(P);
  for (int r = 0; r < P; ++r) {
    XRank<T>& q = R[r];
    q.crd[0] = r / (Pd[1] * Pd[2]);
    q.crd[1] = (r / Pd[2]) % Pd[1];
    q.crd[2] = r % Pd[2];
    for (int a = 0; a < 3; ++a) {
      // near-equal split, the remainder on the first ranks
      const int base = N[a] / Pd[a], rem = N[a] % Pd[a], c = q.crd[a];
      q.lo[a] = c * base + std::min(c, rem);
      q.hi[a] = q.lo[a] + base + (c < rem ? 1 : 0);
      const int gl = c > 0 ? gd[a] : 0, gh = c < Pd[a] - 1 ? gd[a] : 0;
      q.g0[a] = q.lo[a] - gl;
      q.n[a] = q.hi[a] - q.lo[a] + gl + gh;
    }
    if (dim == 3 && (sizeof(T) == 4 || cpml) && q.n[2] % 4 != 0) {
      std::fprintf(stderr, "fdtd3d (native): fp32 / CPML parallel grids need every rank's z extent (ghosts "
                           "included) %% 4 == 0 (4-cell rows): rank %d has %d\n", r, q.n[2]);
      return 2;
    }
  }
  sp = {N[0] / 2, N[1] / 2, N[2] / 2};
  if (scheme == "tmz") sp = {N[0] > 140 ? 70 : N[0] / 2, N[1] / 2, 0};  // (SchemeTMz.cpp:1345)
  if (dim == 1) sp = {N[0] / 2, 0, 0};
  return 0;
}

// one rank on device r % devices: streams, fields, update boxes, the 26
// message boxes and buffers, per-cell coefficients
template <typename T>
void MultiRun<T>::setup_rank(int r) {
  XRank<T>& q = R[r];
  q.dev = r % ndev;
  HIP_OK(hipSetDevice(q.dev));
  HIP_OK(hipStreamCreate(&q.st));
  HIP_OK(hipStreamCreate(&q.side));
  HIP_OK(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
  HIP_OK(hipEventCreateWithFlags(&q.copied, hipEventDisableTiming));
  const size_t n = q.cells();
  for (int c = 0; c < 6; ++c) {
    q.F[c].alloc(n);
    q.G[c].alloc(n);
  }
  // update boxes in local indices: the global range of each component
  // clipped to the rank's allocated box
  for (int c = 0; c < 6; ++c) {
    fdtd::Int3 glo, ghi;
    fdtd::global_range(c, N, active, glo, ghi);
    for (int a = 0; a < 3; ++a) {
      q.boxes[6 * c + a] = std::max(glo[a], q.g0[a]) - q.g0[a];
      q.boxes[6 * c + 3 + a] = std::min(ghi[a], q.g0[a] + q.n[a]) - q.g0[a];
    }
  }
  // messages: direction d = (dx + 1) * 9 + (dy + 1) * 3 + (dz + 1)
  for (int d = 0; d < 27; ++d) {
    const int off[3] = {d / 9 - 1, (d / 3) % 3 - 1, d % 3 - 1};
    int c[3];
    bool ok = d != 13;
    for (int a = 0; a < 3; ++a) {
      c[a] = q.crd[a] + off[a];
      ok = ok && c[a] >= 0 && c[a] < Pd[a];
    }
    // (physics: the face neighbours only -- the split half steps read no
    // diagonal ghost)
    if (phys) ok = ok && std::abs(off[0]) + std::abs(off[1]) + std::abs(off[2]) == 1;
    q.nb[d] = ok ? rank_of(c) : -1;
    if (!ok) continue;
    size_t vol = phys ? 3 : 6;
    for (int a = 0; a < 3; ++a) {
      // send: the owned layers next to the neighbour; receive: the ghosts there
      int slo = q.lo[a], shi = q.hi[a], rlo = q.lo[a], rhi = q.hi[a];
      if (off[a] < 0) {
        shi = q.lo[a] + gd[a];
        rlo = q.lo[a] - gd[a];
        rhi = q.lo[a];
      } else if (off[a] > 0) {
        slo = q.hi[a] - gd[a];
        rlo = q.hi[a];
        rhi = q.hi[a] + gd[a];
      }
      q.sbox[d][a] = slo - q.g0[a];
      q.sbox[d][3 + a] = shi - q.g0[a];
      q.rbox[d][a] = rlo - q.g0[a];
      q.rbox[d][3 + a] = rhi - q.g0[a];
      vol *= (size_t)(shi - slo);
    }
    q.sbuf[d].alloc(vol);
    q.rbuf[d].alloc(vol);
  }
  if (percell) {
    // per-cell E coefficients of the dielectric sphere (2-point eps
    // averages, as the single-rank path; 2D: the cylinder's section at the
    // centre's z), H on the scalar db (2D: db arrays, the 2D kernels take one
    // coefficient form per launch)
    const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
    std::vector<T> host(n);
    for (int c = 0; c < 3; ++c) {
      const int di = c == 0, dj = c == 1, dk = c == 2 && dim == 3;
      for (int li = 0; li < q.n[0]; ++li)
        for (int lj = 0; lj < q.n[1]; ++lj)
          for (int lk = 0; lk < q.n[2]; ++lk) {
            const int i = q.g0[0] + li, j = q.g0[1] + lj, k = q.g0[2] + lk;
            const double z0 = dim == 3 ? k + 0.5 : ctr[2], z1 = dim == 3 ? k + dk + 0.5 : ctr[2];
            const double a = sphere_eps(i + 0.5, j + 0.5, z0, ctr, s.sphereRadius, s.sphereEps);
            const double b = sphere_eps(i + di + 0.5, j + dj + 0.5, z1, ctr, s.sphereRadius, s.sphereEps);
            host[((size_t)li * q.n[1] + lj) * q.n[2] + lk] = (T)(cb * 2.0 / (a + b));
          }
      q.C[c].alloc(n);
      HIP_OK(hipMemcpy(q.C[c].p, host.data(), n * sizeof(T), hipMemcpyHostToDevice));
    }
    if (dim < 3) {
      std::fill(host.begin(), host.end(), (T)db);
      for (int c = 3; c < 6; ++c) {
        q.C[c].alloc(n);
        HIP_OK(hipMemcpy(q.C[c].p, host.data(), n * sizeof(T), hipMemcpyHostToDevice));
      }
    }
  }
}

// peer access between the devices of neighbouring ranks (xGMI)
template <typename T>
void MultiRun<T>::enable_peers() {
  for (int r = 0; r < P; ++r)
    for (int d = 0; d < 27; ++d) {
      const int o = R[r].nb[d];
      if (o < 0 || R[o].dev == R[r].dev) continue;
      int ok = 0;
      HIP_OK(hipDeviceCanAccessPeer(&ok, R[r].dev, R[o].dev));
      if (ok) {
        HIP_OK(hipSetDevice(R[r].dev));
        const hipError_t e = hipDeviceEnablePeerAccess(R[o].dev, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_OK(e);
      }
    }
  (void)hipGetLastError();
}

// output boxes of a pass (local indices): the interior (owned cells at
// least TB from every neighbour: needs no fresh ghost) first, then the
// TB-thick shell slabs peeled off axis by axis (models/blocking.py _tb_regions)
template <typename T>
void MultiRun<T>::plan_outputs() {
  for (XRank<T>& q : R) {
    int lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
      lo[a] = q.lo[a] - q.g0[a];
      hi[a] = q.hi[a] - q.g0[a];
    }
    std::vector<std::array<int, 6>> sh;
    for (int a = 0; a < 3; ++a)
      for (int side = 0; side < 2; ++side) {
        if ((side == 0 ? q.crd[a] == 0 : q.crd[a] == Pd[a] - 1)) continue;
        std::array<int, 6> b = {lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]};
        if (side == 0) {
          b[3 + a] = lo[a] + TB;
          lo[a] += TB;
        } else {
          b[a] = hi[a] - TB;
          hi[a] -= TB;
        }
        sh.push_back(b);
      }
    q.outs.push_back({lo[0], lo[1], lo[2], hi[0], hi[1], hi[2]});
    for (const auto& b : sh) q.outs.push_back(b);
  }
}

// Phase 1 of a pass, every rank on its side stream: pull the neighbours'
// packs of the previous pass (after their `done` and its own, which orders
// the ghost writes after the passes that read them) and unpack them into the
// ghosts
template <typename T>
void MultiRun<T>::pull_ghosts() {
  for (int r = 0; r < P; ++r) {
    XRank<T>& q = R[r];
    HIP_OK(hipSetDevice(q.dev));
    HIP_OK(hipStreamWaitEvent(q.side, q.done, 0));
    T* f[6] = {q.F[0].p, q.F[1].p, q.F[2].p, q.F[3].p, q.F[4].p, q.F[5].p};
    for (int d = 0; d < 27; ++d) {
      if (q.nb[d] < 0) continue;
      const XRank<T>& o = R[q.nb[d]];
      HIP_OK(hipStreamWaitEvent(q.side, o.done, 0));
      // the neighbour at d packed its box for direction 26 - d (towards us)
      const size_t bytes = q.rbuf[d].n * sizeof(T);
      if (o.dev == q.dev)
        HIP_OK(hipMemcpyAsync(q.rbuf[d].p, o.sbuf[26 - d].p, bytes, hipMemcpyDeviceToDevice, q.side));
      else
        HIP_OK(hipMemcpyPeerAsync(q.rbuf[d].p, q.dev, o.sbuf[26 - d].p, o.dev, bytes, q.side));
      K_OK(box_unpack(f, q.rbuf[d].p, 6, q.n[1], q.n[2], q.rbox[d], q.side));
    }
    HIP_OK(hipEventRecord(q.copied, q.side));
  }
}

// Phase 2 for one rank, on its main stream: the interior -- concurrent with
// phase 1, it reads no ghost -- then, after the pulls, the shells, and the
// packs for the next pass once the neighbours have pulled this pass's (their
// `copied`)
template <typename T>
void MultiRun<T>::rank_pass(XRank<T>& q, int t, int k) {
  HIP_OK(hipSetDevice(q.dev));
  const T* ei[3] = {q.F[0].p, q.F[1].p, q.F[2].p};
  const T* hi[3] = {q.F[3].p, q.F[4].p, q.F[5].p};
  T* eo[3] = {q.G[0].p, q.G[1].p, q.G[2].p};
  T* ho[3] = {q.G[3].p, q.G[4].p, q.G[5].p};
  const T* cbs[3] = {q.C[0].p, q.C[1].p, q.C[2].p};
  const T* dbs[3] = {nullptr, nullptr, nullptr};
  // every rank whose allocated box (ghosts included) holds the source
  // sets the hard source: a neighbour's redundant ghost levels need it
  bool has = true;
  for (int a = 0; a < 3; ++a) has = has && sp[a] >= q.g0[a] && sp[a] < q.g0[a] + q.n[a];
  const int src[4] = {sp[0] - q.g0[0], sp[1] - q.g0[1], sp[2] - q.g0[2], has ? 2 : -1};
  double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int l = 0; l < k; ++l) vals[l] = src_val(t + l);
  for (size_t b = 0; b < q.outs.size(); ++b) {
    const int* ob = q.outs[b].data();
    if (b == 1 && !first) HIP_OK(hipStreamWaitEvent(q.st, q.copied, 0));  // the shells read the fresh ghosts
    if (ob[3] <= ob[0] || ob[4] <= ob[1] || ob[5] <= ob[2]) continue;
    if constexpr (sizeof(T) == 4)
      K_OK(fdtd_tb3d_v4_f32(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, db, q.n[0], q.n[1], q.n[2], q.boxes, ob, 0,
                            k, src, vals, q.st));
    else
      K_OK(fdtd_tb3d_f64(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, db, q.n[0], q.n[1], q.n[2], q.boxes, ob, 0, k,
                         src, vals, q.st));
  }
  if (!first && q.outs.size() == 1) HIP_OK(hipStreamWaitEvent(q.st, q.copied, 0));  // a lone rank
  for (int c = 0; c < 6; ++c) std::swap(q.F[c].p, q.G[c].p);
  // the neighbours have pulled the previous packs before these overwrite them
  if (!first)
    for (int d = 0; d < 27; ++d)
      if (q.nb[d] >= 0) HIP_OK(hipStreamWaitEvent(q.st, R[q.nb[d]].copied, 0));
  T* f[6] = {q.F[0].p, q.F[1].p, q.F[2].p, q.F[3].p, q.F[4].p, q.F[5].p};
  for (int d = 0; d < 27; ++d)
    if (q.nb[d] >= 0) K_OK(box_pack(f, q.sbuf[d].p, 6, q.n[1], q.n[2], q.sbox[d], q.st));
  HIP_OK(hipEventRecord(q.done, q.st));
}

// One pass of k steps: the phases are issued rank after rank on the host, so
// every event waited on is already recorded.
template <typename T>
void MultiRun<T>::pass(int t, int k) {
  if (!first) pull_ghosts();
  for (int r = 0; r < P; ++r) rank_pass(R[r], t, k);
  first = false;
}

// UPML / Drude tables of a rank at the global positions, and its part of the
// global chain regions (the PML slabs with one cell of staggering slack, the
// dispersive sphere's box; native_run.h setup_chain_regions) with their
// region-local D / D1 levels
template <typename T>
void MultiRun<T>::setup_chain(XRank<T>& q) {
  native_phys::UpmlScene sc;
  sc.pml[0] = s.pmlSizeX;
  sc.pml[1] = s.pmlSizeY;
  sc.pml[2] = s.pmlSizeZ;
  sc.use_pml = s.doUsePML;
  sc.metamaterials = s.doUseMetamaterials;
  sc.lorentz = s.dispersion == "lorentz";
  sc.lorentz_ratio = s.lorentzOmega0Ratio;
  sc.freq = freq;
  sc.sphere_eps = s.scene == "sphere";
  sc.drude_sphere = s.scene == "drude-sphere";
  sc.ctr[0] = s.sphereCenterX;
  sc.ctr[1] = s.sphereCenterY;
  sc.ctr[2] = s.sphereCenterZ;
  sc.radius = s.sphereRadius;
  sc.eps_in = s.sphereEps;
  q.up.reset(new native_phys::Upml<T>());
  native_phys::setup_upml<T>(*q.up, N, sc, dt, s.gridStep, q.g0, q.n, true);
  // the global regions
  const IBox whole_box = {{0, 0, 0}, {N[0], N[1], N[2]}};
  const int pp[3] = {s.doUsePML ? s.pmlSizeX + 1 : 0, s.doUsePML ? s.pmlSizeY + 1 : 0,
                     s.doUsePML ? s.pmlSizeZ + 1 : 0};
  const IBox inner = {{pp[0], pp[1], pp[2]}, {N[0] - pp[0], N[1] - pp[1], N[2] - pp[2]}};
  IBox dbox = {{0, 0, 0}, {0, 0, 0}};
  if (s.doUseMetamaterials)
    for (int a = 0; a < 3; ++a) {
      dbox.lo[a] = std::max(0, (int)std::floor(sc.ctr[a] - s.sphereRadius) - 2);
      dbox.hi[a] = std::min(N[a], (int)std::ceil(sc.ctr[a] + s.sphereRadius) + 3);
    }
  bool inside = !inner.empty();
  for (int a = 0; a < 3 && !dbox.empty(); ++a) inside = inside && dbox.lo[a] >= inner.lo[a] && dbox.hi[a] <= inner.hi[a];
  std::vector<IBox> creg, preg;
  std::vector<bool> cdisp;
  if (!inside) {
    creg.push_back(whole_box);
    cdisp.push_back(true);
  } else {
    if (s.doUsePML) creg = box_minus(whole_box, inner);
    cdisp.assign(creg.size(), false);
    if (!dbox.empty()) {
      creg.push_back(dbox);
      cdisp.push_back(true);
      preg = box_minus(inner, dbox);
    } else {
      preg.push_back(inner);
    }
  }
  // the rank's parts, local indices
  const IBox own = {{q.lo[0], q.lo[1], q.lo[2]}, {q.hi[0], q.hi[1], q.hi[2]}};
  auto local = [&](const IBox& b) {
    IBox r = box_and(b, own);
    for (int a = 0; a < 3; ++a) {
      r.lo[a] -= q.g0[a];
      r.hi[a] -= q.g0[a];
    }
    return r;
  };
  std::vector<std::array<int, 6>> rb;
  for (size_t r = 0; r < creg.size(); ++r) {
    const IBox b = local(creg[r]);
    if (b.empty()) continue;
    q.chain_regs.push_back(b);
    q.chain_disp.push_back(cdisp[r]);
    rb.push_back({b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2]});
  }
  for (const IBox& p : preg) {
    const IBox b = local(p);
    if (!b.empty()) q.plain_regs.push_back(b);
  }
  native_phys::alloc_levels(*q.up, rb, q.chain_disp);
}

// the component boxes (36 ints) clipped to a region
template <typename T>
void MultiRun<T>::clip36(const int* b36, const IBox& r, int* out) {
  for (int c = 0; c < 6; ++c) {
    IBox b;
    for (int a = 0; a < 3; ++a) {
      b.lo[a] = b36[6 * c + a];
      b.hi[a] = b36[6 * c + 3 + a];
    }
    b = box_and(b, r);
    for (int a = 0; a < 3; ++a) {
      out[6 * c + a] = b.empty() ? 0 : b.lo[a];
      out[6 * c + 3 + a] = b.empty() ? 0 : b.hi[a];
    }
  }
}

// amplitude mode of a rank (native_amp.h AmpMode on the rank's cells): the
// maxima and counts, each component's amplitude box (its update range minus
// the PML cells, Scheme3D.cpp:3016-3030) clipped to the owned cells, the owned
// cells of the Ez z line at (Nx / 8, Ny / 2) outside the z PML (Scheme3D.cpp:2995-3013)
template <typename T>
void MultiRun<T>::setup_amp(XRank<T>& q) {
  const size_t plane = (size_t)q.n[1] * q.n[2];
  q.AMP.alloc((size_t)q.n[0] * 6 * plane);
  q.CNT.alloc(std::max(1, s.amplitudeCheckSteps));
  const int left[3] = {s.doUsePML ? s.pmlSizeX : 0, s.doUsePML ? s.pmlSizeY : 0, s.doUsePML ? s.pmlSizeZ : 0};
  for (int c = 0; c < 6; ++c) {
    fdtd::Int3 glo, ghi;
    fdtd::global_range(c, N, active, glo, ghi);
    int* b = q.ab + 6 * c;
    bool empty = false;
    for (int a = 0; a < 3; ++a) {
      int lo = glo[a], hi = ghi[a];
      const int right = N[a] - left[a];
      const bool act = std::find(active.begin(), active.end(), a) != active.end();
      if (act && left[a] != right) {
        lo = std::max(lo, (int)std::ceil(left[a] - kMinFP[c][a]));
        hi = std::min(hi, (int)std::ceil(right - kMinFP[c][a]));
      }
      lo = std::max(lo, q.lo[a]);
      hi = std::min(hi, q.hi[a]);
      empty = empty || hi <= lo;
      b[a] = lo - q.g0[a];
      b[3 + a] = hi - q.g0[a];
    }
    if (empty || !present[c])
      for (int e = 0; e < 6; ++e) b[e] = 0;
  }
  amp_line = point_src && dim == 3;  // (2D: the point source stays)
  if (!amp_line) return;
  const int k0 = s.doUsePML ? s.pmlSizeZ : 0;
  amp_line = N[2] - 2 * k0 > 0;
  const int li = N[0] / 8, lj = N[1] / 2;
  std::vector<long long> offs;
  if (li >= q.lo[0] && li < q.hi[0] && lj >= q.lo[1] && lj < q.hi[1])
    for (int k = std::max(k0, q.lo[2]); k < std::min(N[2] - k0, q.hi[2]); ++k)
      offs.push_back(((long long)(li - q.g0[0]) * q.n[1] + (lj - q.g0[1])) * q.n[2] + (k - q.g0[2]));
  q.line_n = (int)offs.size();
  if (q.line_n > 0) {
    q.LINE.alloc(offs.size());
    HIP_OK(hipMemcpy(q.LINE.p, offs.data(), offs.size() * sizeof(long long), hipMemcpyHostToDevice));
  }
}

// every array of a rank that carries state between steps (the amplitude
// phase's near-convergence snapshot; native_run.h amp_state)
template <typename T>
std::vector<std::pair<void*, size_t>> MultiRun<T>::rank_state(XRank<T>& q) {
  std::vector<std::pair<void*, size_t>> v;
  for (int c = 0; c < 6; ++c) v.push_back({q.F[c].p, q.cells() * sizeof(T)});
  v.push_back({q.AMP.p, q.AMP.n * sizeof(T)});
  if (q.tf) {
    v.push_back({q.tf->einc.p, (size_t)q.tf->nline * sizeof(T)});
    v.push_back({q.tf->hinc.p, (size_t)q.tf->nline * sizeof(T)});
  }
  if (q.cp)
    for (auto* d : q.cp->keep) v.push_back({d->p, d->n * sizeof(T)});
  if (q.p2) {
    for (const Slab2d<T>& sl : q.p2->slabs)
      v.push_back({sl.psi, (size_t)(sl.pbox[3] - sl.pbox[0]) * (sl.pbox[4] - sl.pbox[1]) * (sl.pbox[5] - sl.pbox[2]) *
                               sizeof(T)});
    for (int c = 0; c < 6; ++c)
      for (int l = 0; l < 2; ++l)
        if (q.p2->D[c][l]) v.push_back({q.p2->D[c][l], q.cells() * sizeof(T)});
  }
  if (q.up)
    for (int c = 0; c < 6; ++c) {
      for (const auto& lv : q.up->D[c])
        for (size_t r = 0; r < lv.size(); ++r) v.push_back({lv[r], q.up->rvol[r] * sizeof(T)});
      for (const auto& lv : q.up->D1[c])
        for (size_t r = 0; r < lv.size(); ++r)
          if (lv[r]) v.push_back({lv[r], q.up->rvol[r] * sizeof(T)});
    }
  return v;
}

// The amplitude phase from step t over the ranks (native_amp.h AmpMode::run):
// check periods of K steps, each step's changed-maximum counts summed over
// the ranks once per period; the run ends with the period in which a step
// (after the first) changed no maximum -- redone from a snapshot up to that
// step near convergence -- or after --amplitude-time-steps steps.  Returns
// the last step.
template <typename T>
int MultiRun<T>::amp_run(int t) {
  amp_on = true;
  const int K = std::max(1, s.amplitudeCheckSteps);
  std::vector<unsigned> got(K), part(K);
  auto period = [&](int n) {
    for (XRank<T>& q : R) {
      HIP_OK(hipSetDevice(q.dev));
      HIP_OK(hipMemsetAsync(q.CNT.p, 0, K * sizeof(unsigned), q.st));
    }
    for (int i = 0; i < n; ++i) {
      phys_step(t);
      for (XRank<T>& q : R) {
        HIP_OK(hipSetDevice(q.dev));
        const T* af[6] = {q.F[0].p, q.F[1].p, q.F[2].p, q.F[3].p, q.F[4].p, q.F[5].p};
        const size_t plane = (size_t)q.n[1] * q.n[2];
        T* aa[6];
        for (int c = 0; c < 6; ++c) aa[c] = q.AMP.p + c * plane;
        K_OK(amp_many(af, aa, 6, q.n[1], q.n[2], q.ab, (long long)(6 * plane), 0.001, q.CNT.p + i, q.st));
      }
      ++t;
    }
    std::fill(got.begin(), got.end(), 0u);
    for (XRank<T>& q : R) {
      HIP_OK(hipSetDevice(q.dev));
      HIP_OK(hipMemcpyAsync(part.data(), q.CNT.p, n * sizeof(unsigned), hipMemcpyDeviceToHost, q.st));
      HIP_OK(hipStreamSynchronize(q.st));
      for (int i = 0; i < n; ++i) got[i] += part[i];
    }
  };
  long long acells = 0;
  for (XRank<T>& q : R)
    for (int c = 0; c < 6; ++c) {
      const int* b = q.ab + 6 * c;
      acells += (long long)std::max(0, b[3] - b[0]) * std::max(0, b[4] - b[1]) * std::max(0, b[5] - b[2]);
    }
  const long long near = std::max(1LL, (long long)(0.02 * (double)acells));
  long long last = -1;
  bool done = false;
  while (!done && amp_taken < s.numAmplitudeTimeSteps) {
    int n = std::min(K, s.numAmplitudeTimeSteps - amp_taken);
    int t_snap = -1;
    if (n > 1 && last >= 0 && last <= near) {
      for (XRank<T>& q : R) {
        HIP_OK(hipSetDevice(q.dev));
        const auto v = rank_state(q);
        size_t total = 0, o = 0;
        for (const auto& e : v) total += e.second;
        if (!q.SNAP.p) q.SNAP.alloc(total);
        for (const auto& e : v) {
          HIP_OK(hipMemcpyAsync(q.SNAP.p + o, e.first, e.second, hipMemcpyDeviceToDevice, q.st));
          o += e.second;
        }
      }
      t_snap = t;
    }
    period(n);
    int first = -1;
    for (int r = 0; r < n && first < 0; ++r)
      if (got[r] == 0 && amp_taken + r + 1 > 1) first = r;
    if (first < 0) {
      last = got[n - 1];
      amp_taken += n;
      continue;
    }
    amp_stable = amp_taken + first + 1;
    if (first + 1 < n && t_snap >= 0) {
      for (XRank<T>& q : R) {
        HIP_OK(hipSetDevice(q.dev));
        const auto v = rank_state(q);
        size_t o = 0;
        for (const auto& e : v) {
          HIP_OK(hipMemcpyAsync(e.first, q.SNAP.p + o, e.second, hipMemcpyDeviceToDevice, q.st));
          o += e.second;
        }
      }
      t = t_snap;
      n = first + 1;
      period(n);
    }
    amp_taken += n;
    done = true;
  }
  amp_on = false;
  return t;
}

// physics set-up of rank r (its device current): owned update boxes, CPML
// tables, TF/SF tables and incident line, the point source; false when the
// TF/SF box does not fit the incident line
template <typename T>
bool MultiRun<T>::setup_physics(int r) {
  XRank<T>& q = R[r];
  int own[6], gb36[36];
  for (int a = 0; a < 3; ++a) {
    own[a] = q.lo[a];
    own[3 + a] = q.hi[a];
  }
  for (int c = 0; c < 6; ++c) {
    fdtd::Int3 glo, ghi;
    fdtd::global_range(c, N, active, glo, ghi);
    bool empty = false;
    for (int a = 0; a < 3; ++a) {
      const int lo = std::max(glo[a], q.lo[a]), hi = std::min(ghi[a], q.hi[a]);
      empty = empty || hi <= lo;
      gb36[6 * c + a] = lo;
      gb36[6 * c + 3 + a] = hi;
    }
    for (int a = 0; a < 3; ++a) {
      if (empty) gb36[6 * c + a] = gb36[6 * c + 3 + a] = 0;
      q.own36[6 * c + a] = empty ? 0 : gb36[6 * c + a] - q.g0[a];
      q.own36[6 * c + 3 + a] = empty ? 0 : gb36[6 * c + 3 + a] - q.g0[a];
    }
  }
  if (dim == 2) {
    q.p2.reset(new Pml2d<T>());
    if (cpml) setup_cpml2d(*q.p2, s, N, active, present, dt, s.gridStep, own, q.g0, q.n);
    if (upml) {
      // per-cell 1 / (eps eps0) of a dielectric scene (E components), as native_run.h setup_absorbers
      std::vector<T> inv[3];
      if (percell) {
        const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
        for (int c = 0; c < 3; ++c) {
          if (!present[c]) continue;
          inv[c].resize(q.cells());
          const int di = c == 0, dj = c == 1;
          for (int li = 0; li < q.n[0]; ++li)
            for (int lj = 0; lj < q.n[1]; ++lj) {
              const int i = q.g0[0] + li, j = q.g0[1] + lj;
              const double a = sphere_eps(i + 0.5, j + 0.5, ctr[2], ctr, s.sphereRadius, s.sphereEps);
              const double b = sphere_eps(i + di + 0.5, j + dj + 0.5, ctr[2], ctr, s.sphereRadius, s.sphereEps);
              inv[c][(size_t)li * q.n[1] + lj] = (T)(1.0 / ((a + b) / 2.0 * kEps0));
            }
        }
      }
      setup_upml2d(*q.p2, s, N, present, dt, s.gridStep, inv, q.g0, q.n);
    }
    const fdtd::Int3 ext = {q.n[0], q.n[1], q.n[2]};
    q.ld.reset(new Lowdim2d<T>(s, q.F, q.C, q.own36, ext, present, *q.p2, scheme == "tmz", percell, cb, db, q.st, &N,
                               q.g0));
  } else {
    if (cpml) {
      q.cp.reset(new NativeCpml<T>());
      setup_cpml(*q.cp, s, N, active, dt, s.gridStep, own, q.g0, q.n);
    }
    if (upml) setup_chain(q);
  }
  if (tfsf) {
    q.tf.reset(new NativeTfsf<T>());
    // (E: per-cell arrays of the sphere or the scalar; H: the scalar db, mu = 1 -- 1D / 2D: db arrays)
    if (!setup_tfsf(*q.tf, s, N, gb36, q.C, percell ? 1.0 : cb, dim < 3 && percell ? 1.0 : db, dt, s.gridStep, freq,
                    dim, present, q.g0, q.n))
      return false;
  }
  if (amp) setup_amp(q);
  bool has = point_src;
  for (int a = 0; a < 3; ++a) has = has && sp[a] >= q.lo[a] && sp[a] < q.hi[a];
  q.src_off = has ? ((long long)(sp[0] - q.g0[0]) * q.n[1] + (sp[1] - q.g0[1])) * q.n[2] + (sp[2] - q.g0[2]) : -1;
  return true;
}

// one half step of one rank on its main stream, the order of the single-GPU
// stepped path (native_run.h step3d_split): [incident line] update (+ CPML
// psi) [TF/SF corrections] [point source, E]
template <typename T>
void MultiRun<T>::phys_half(XRank<T>& q, int kind, double sv) {
  HIP_OK(hipSetDevice(q.dev));
  T* F[6] = {q.F[0].p, q.F[1].p, q.F[2].p, q.F[3].p, q.F[4].p, q.F[5].p};
  const T* C[6] = {q.C[0].p, q.C[1].p, q.C[2].p, nullptr, nullptr, nullptr};
  const bool v4 = sizeof(T) == 4 && q.n[2] % 4 == 0;
  if (tfsf) {
    NativeTfsf<T>& tf = *q.tf;
    if (kind == 0)
      K_OK(inc_e(tf.einc.p, tf.hinc.p, tf.nline, tf.ce, sv, q.st));
    else
      K_OK(inc_h(tf.einc.p, tf.hinc.p, tf.nline, tf.ch, q.st));
  }
  const int* bx = q.own36 + 18 * kind;
  if (dim == 1) {
    // native_run.h step: the 1D Ez / Hy kernels over the owned x range
    if (kind == 0)
      K_OK(e1d(F[2], F[4], C[2], percell ? 1.0 : cb, q.own36[12], q.own36[15], q.st));
    else
      K_OK(h1d(F[4], F[2], q.C[4].p, percell ? 1.0 : db, q.own36[24], q.own36[27], q.st));
  } else if (dim == 2) {
    // native_run.h step2d: the plain 2D kernels (or the UPML chain on the
    // strips + the plain kernels inside), then the CPML corrections
    const IBox all = {{0, 0, 0}, {q.n[0], q.n[1], q.n[2]}};
    if (upml)
      q.ld->upml(kind);
    else
      q.ld->plain(kind, all);
    if (cpml) q.ld->cpml(kind);
  } else if (upml) {
    // the chain on the rank's part of the PML slabs and the dispersive box,
    // the plain update on the rest (native_run.h upml_regions)
    using ChainFn = int (*)(const void* const*, const double*, const int*, int, int, int, int, void*);
    const ChainFn chain = sizeof(T) == 4 ? (ChainFn)fdtd_chain3d_f32 : (ChainFn)fdtd_chain3d_f64;
    int rb[36];
    for (size_t r = 0; r < q.chain_regs.size(); ++r) {
      clip36(q.own36, q.chain_regs[r], rb);
      K_OK(native_phys::upml_kind<T>(*q.up, F, rb, kind, q.n[1], q.n[2], q.st, chain, false, !q.chain_disp[r], nullptr,
                                     1.0, (int)r));
    }
    native_phys::upml_rotate(*q.up, kind);
    for (const IBox& pr : q.plain_regs) {
      clip36(q.own36, pr, rb);
      if (kind == 0)
        K_OK(e3d(F[0], F[1], F[2], F[3], F[4], F[5], C[0], C[1], C[2], percell ? 1.0 : cb, q.n[0], q.n[1], q.n[2], rb,
                 0, q.st, v4));
      else
        K_OK(h3d(F[3], F[4], F[5], F[0], F[1], F[2], nullptr, nullptr, nullptr, db, q.n[0], q.n[1], q.n[2], rb + 18,
                 0, q.st, v4));
    }
  } else if (kind == 0) {
    if (cpml)
      K_OK(cpml_e3d(F, C, percell ? 1.0 : cb, q.n[0], q.n[1], q.n[2], q.own36, q.cp->P[0].data(), q.cp->I[0].data(),
                    q.st));
    else
      K_OK(e3d(F[0], F[1], F[2], F[3], F[4], F[5], C[0], C[1], C[2], percell ? 1.0 : cb, q.n[0], q.n[1], q.n[2], bx,
               0, q.st, v4));
  } else {
    if (cpml)
      K_OK(cpml_h3d(F, C, db, q.n[0], q.n[1], q.n[2], bx, q.cp->P[1].data(), q.cp->I[1].data(), q.st));
    else
      K_OK(h3d(F[3], F[4], F[5], F[0], F[1], F[2], nullptr, nullptr, nullptr, db, q.n[0], q.n[1], q.n[2], bx, 0, q.st,
               v4));
  }
  if (tfsf) {
    const int whole[6] = {0, 0, 0, q.n[0], q.n[1], q.n[2]};
    for (int c = 3 * kind; c < 3 * kind + 3; ++c)
      for (auto* l : q.tf->tab[c])
        K_OK(tfsf_apply(F[c], *l, kind == 0 ? q.tf->hinc.p : q.tf->einc.p, whole, q.st));
  }
  if (kind == 0) {
    if (amp_on && amp_line) {  // the amplitude phase's Ez z line replaces the point source
      if (q.line_n > 0) K_OK(setvs(F[2], q.LINE.p, q.line_n, sv, q.st));
    } else if (q.src_off >= 0) {
      K_OK(setv(F[src_comp], q.src_off, sv, q.st));
    }
  }
}

// the updated kind's three components to the face neighbours' ghosts: every
// rank packs its boxes (after the neighbours pulled the previous ones), then
// every rank pulls (peer copies across devices) and unpacks on its main
// stream, so its next half step reads the fresh ghosts
template <typename T>
void MultiRun<T>::exchange(int kind) {
  for (int r = 0; r < P; ++r) {
    XRank<T>& q = R[r];
    HIP_OK(hipSetDevice(q.dev));
    T* f[3] = {q.F[3 * kind].p, q.F[3 * kind + 1].p, q.F[3 * kind + 2].p};
    for (int d = 0; d < 27; ++d) {
      if (q.nb[d] < 0) continue;
      if (!first) HIP_OK(hipStreamWaitEvent(q.st, R[q.nb[d]].copied, 0));
      K_OK(box_pack(f, q.sbuf[d].p, 3, q.n[1], q.n[2], q.sbox[d], q.st));
    }
    HIP_OK(hipEventRecord(q.done, q.st));
  }
  for (int r = 0; r < P; ++r) {
    XRank<T>& q = R[r];
    HIP_OK(hipSetDevice(q.dev));
    T* f[3] = {q.F[3 * kind].p, q.F[3 * kind + 1].p, q.F[3 * kind + 2].p};
    for (int d = 0; d < 27; ++d) {
      if (q.nb[d] < 0) continue;
      const XRank<T>& o = R[q.nb[d]];
      HIP_OK(hipStreamWaitEvent(q.st, o.done, 0));
      const size_t bytes = q.rbuf[d].n * sizeof(T);
      if (o.dev == q.dev)
        HIP_OK(hipMemcpyAsync(q.rbuf[d].p, o.sbuf[26 - d].p, bytes, hipMemcpyDeviceToDevice, q.st));
      else
        HIP_OK(hipMemcpyPeerAsync(q.rbuf[d].p, q.dev, o.sbuf[26 - d].p, o.dev, bytes, q.st));
      K_OK(box_unpack(f, q.rbuf[d].p, 3, q.n[1], q.n[2], q.rbox[d], q.st));
    }
    HIP_OK(hipEventRecord(q.copied, q.st));
  }
  first = false;
}

template <typename T>
void MultiRun<T>::phys_step(int t) {
  const double sv = src_val(t);
  for (int kind = 0; kind < 2; ++kind) {
    for (int r = 0; r < P; ++r) phys_half(R[r], kind, sv);
    if (P > 1) exchange(kind);
  }
}

template <typename T>
void MultiRun<T>::advance(int t0, int n) {
  if (phys) {
    for (int q = 0; q < n; ++q) phys_step(t0 + q);
    return;
  }
  int t = t0;
  while (n > 0) {
    const int k = std::min(TB, n);
    pass(t, k);
    t += k;
    n -= k;
  }
}

template <typename T>
void MultiRun<T>::sync_all() {
  for (int r = 0; r < P; ++r) {
    HIP_OK(hipSetDevice(R[r].dev));
    HIP_OK(hipStreamSynchronize(R[r].st));
  }
}

template <typename T>
void MultiRun<T>::report(double sec, int t_end, int steps, int warm) const {
  const double cells = (double)N[0] * N[1] * N[2];
  const int timed = steps - warm + amp_taken;
  std::printf("Total time = %f seconds\n", sec);
  std::printf("Dimension: %d\n", dim);
  if (dim == 3)
    std::printf("Grid size: %dx%dx%d\n", N[0], N[1], N[2]);
  else if (dim == 2)
    std::printf("Grid size: %dx%d\n", N[0], N[1]);
  else
    std::printf("Grid size: %d\n", N[0]);
  std::printf("Number of time steps: %d (%d timed after %d warm-up)\n\n", t_end, timed, warm);
  std::printf("Value type: %s\n", Api<T>::name);
  std::printf("\n-------- Details --------\n");
  std::printf("Parallel grid: 1\n");
  std::printf("Number of processes: %d (ranks of one process on %d device%s)\n", P, std::min(P, ndev),
              std::min(P, ndev) > 1 ? "s" : "");
  std::string scheme;
  for (int a = 0; a < 3; ++a)
    if (Pd[a] > 1) scheme += "XYZ"[a];
  std::printf("Parallel grid scheme: %s (topology %dx%dx%d)\n", scheme.empty() ? "X" : scheme.c_str(), Pd[0], Pd[1],
              Pd[2]);
  std::printf("Buffer size: %d\n", TB);
  if (phys)
    std::printf("Backend: native HIP, split half-step kernels (%s%s%s), face ghosts (%d x / %d y / %d z cells) by "
                "packed peer copies after every half step\n",
                cpml ? "CPML" : (upml ? (s.doUseMetamaterials ? "UPML D/B chain + dispersive sphere" : "UPML D/B chain")
                                      : (tfsf ? "" : (dim == 3 ? "plain" : (dim == 2 ? "2D" : "1D")))),
                (cpml || upml) && tfsf ? " + " : "", tfsf ? "TF/SF" : "", gd[0], gd[1], gd[2]);
  else
    std::printf("Backend: native HIP, temporally blocked kernel (%d steps per pass), 26-neighbour ghost boxes by "
                "packed peer copies\n", TB);
  std::printf("Throughput: %.1f Mcells/s\n", cells * timed / sec / 1e6);
  if (amp) {
    if (amp_stable > 0)
      std::printf("Amplitude mode: stable after %d steps (%d amplitude steps taken)\n", amp_stable, amp_taken);
    else
      std::printf("Amplitude mode: stable state not reached after %d steps\n", amp_taken);
  }
  if (s.doPrintJson)
    std::printf("{\"seconds\": %.6f, \"steps\": %d, \"mcells_per_s\": %.3f, \"ranks\": %d}\n", sec, timed,
                cells * timed / sec / 1e6, P);
}

// component c of the whole grid on the host: every rank's owned block
template <typename T>
void MultiRun<T>::gather(int c, std::vector<T>& host) {
  host.resize((size_t)N[0] * N[1] * N[2]);
  std::vector<T> loc;
  for (int r = 0; r < P; ++r) {
    const XRank<T>& q = R[r];
    HIP_OK(hipSetDevice(q.dev));
    loc.resize(q.cells());
    HIP_OK(hipMemcpy(loc.data(), q.F[c].p, loc.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (int i = q.lo[0]; i < q.hi[0]; ++i)
      for (int j = q.lo[1]; j < q.hi[1]; ++j)
        std::memcpy(host.data() + ((size_t)i * N[1] + j) * N[2] + q.lo[2],
                    loc.data() + ((size_t)(i - q.g0[0]) * q.n[1] + (j - q.g0[1])) * q.n[2] + (q.lo[2] - q.g0[2]),
                    (size_t)(q.hi[2] - q.lo[2]) * sizeof(T));
  }
}

// the NTFF scattered power diagram of step t (native_run.h ntff_report): the
// ranks' owned blocks assembled into whole-grid arrays on the first rank's
// device, then the one-GPU surface reduction
template <typename T>
void MultiRun<T>::ntff_report(int t) {
  sync_all();
  std::vector<T> host;
  T* Fp[6];
  for (int c = 0; c < 6; ++c) {
    gather(c, host);
    HIP_OK(hipSetDevice(R[0].dev));
    if (!NG[c].p) NG[c].alloc(host.size());
    HIP_OK(hipMemcpy(NG[c].p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
    Fp[c] = NG[c].p;
  }
  const int nbox[3] = {s.ntffSizeX, s.ntffSizeY, s.ntffSizeZ};
  const std::vector<double> phis = native_phys::reference_angles();
  const std::vector<double> p = native_phys::ntff_power<T>(Fp, N, nbox, s.gridStep, s.sourceWaveLength,
                                                           s.incidentWaveAngle1 * (kPi / 180.0), phis);
  for (size_t q = 0; q < phis.size(); ++q)
    std::printf("=== t=%u, inc angle=%f; angle %f === %.17g \n", (unsigned)t, s.incidentWaveAngle2 * (kPi / 180.0),
                phis[q], p[q]);
}

// the steps, with the NTFF diagram after every step t with (t - 1) % ntffStep
// == 0 (native_run.h run_steps)
template <typename T>
void MultiRun<T>::run_steps(int t0, int n) {
  if (!ntff) {
    advance(t0, n);
    return;
  }
  const int nstep = std::max(1, s.ntffStep);
  int t = t0;
  const int end = t0 + n;
  while (t < end) {
    const int nxt = std::min(end, t + 1 + ((1 - (t + 1)) % nstep + nstep) % nstep);
    advance(t, nxt - t);
    t = nxt;
    if ((t - 1) % nstep == 0) ntff_report(t - 1);
  }
}

// component c of the whole grid into every rank's allocated box (owned cells
// and ghosts: a resumed run's first pass reads the ghosts as they are)
template <typename T>
void MultiRun<T>::scatter(int c, const std::vector<T>& host) {
  std::vector<T> loc;
  for (int r = 0; r < P; ++r) {
    XRank<T>& q = R[r];
    loc.resize(q.cells());
    for (int li = 0; li < q.n[0]; ++li)
      for (int lj = 0; lj < q.n[1]; ++lj)
        std::memcpy(loc.data() + ((size_t)li * q.n[1] + lj) * q.n[2],
                    host.data() + ((size_t)(q.g0[0] + li) * N[1] + (q.g0[1] + lj)) * N[2] + q.g0[2],
                    (size_t)q.n[2] * sizeof(T));
    HIP_OK(hipSetDevice(q.dev));
    HIP_OK(hipMemcpy(q.F[c].p, loc.data(), loc.size() * sizeof(T), hipMemcpyHostToDevice));
  }
}

// --checkpoint-step P: a checkpoint after every step t with t % P == 0 (the
// gathered grid in the serial form, native_ckpt.h; its I/O time is kept out
// of the reported rate as in native_run.h run_ckpt)
template <typename T>
void MultiRun<T>::run_ckpt(int t, int n) {
  const int Pc = s.checkpointDir.empty() ? 0 : s.checkpointStep;
  if (Pc <= 0) {
    run_steps(t, n);
    return;
  }
  const int end = t + n;
  while (t < end) {
    const int nxt = std::min(end, (t / Pc + 1) * Pc);
    run_steps(t, nxt - t);
    t = nxt;
    if (t % Pc == 0) {
      sync_all();
      const auto c0 = std::chrono::steady_clock::now();
      if (!ckpt_save<T>(s, scheme, N, present, [this](int c, std::vector<T>& host) { gather(c, host); }, t,
                        s.gridStep, dt)) {
        std::fprintf(stderr, "fdtd3d: cannot write the checkpoint to %s\n", s.checkpointDir.c_str());
        std::exit(1);
      }
      ckpt_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
    }
  }
}

// --save-res: the owned blocks of every rank assembled into global DAT / BMP
// files; --checkpoint-dir: the final checkpoint (gathered, serial form)
template <typename T>
bool MultiRun<T>::save_results(int steps) {
  if (!s.checkpointDir.empty()) {
    if (!ckpt_save<T>(s, scheme, N, present, [this](int c, std::vector<T>& host) { gather(c, host); }, steps,
                      s.gridStep, dt)) {
      std::fprintf(stderr, "fdtd3d: cannot write the checkpoint to %s\n", s.checkpointDir.c_str());
      return false;
    }
  }
  if (!s.doSaveRes) return true;
  const char* names[6] = {"Ex", "Ey", "Ez", "Hx", "Hy", "Hz"};
  std::vector<T> host;
  for (int c = 0; c < 6; ++c) {
    if (!present[c]) continue;
    gather(c, host);
    const std::string base = fdtd::grid_file_name(steps, 0, names[c], s.outputDir == "." ? "" : s.outputDir);
    if (s.saveAsDAT) fdtd::write_dat(base + ".dat", host.data(), host.size() * sizeof(T));
    if (s.saveAsBMP || !s.saveAsDAT) {
      const int kz = dim == 3 ? N[2] / 2 : 0;
      std::vector<double> v((size_t)N[0] * N[1]);
      for (int i = 0; i < N[0]; ++i)
        for (int j = 0; j < N[1]; ++j) v[(size_t)i * N[1] + j] = host[((size_t)i * N[1] + j) * N[2] + kz];
      fdtd::write_bmp(dim == 3 ? base + std::to_string(kz) + "-Re.bmp" : base + "-Re.bmp", v, N[0], N[1],
                      s.dumperPalette);
    }
  }
  return true;
}

template <typename T>
void MultiRun<T>::release() {
  for (auto& q : R) {
    if (!q.st) continue;
    HIP_OK(hipSetDevice(q.dev));
    for (int c = 0; c < 6; ++c) {  // freed with the rank's device current
      q.F[c].reset();
      q.G[c].reset();
      q.C[c].reset();
    }
    for (int d = 0; d < 27; ++d) {
      q.sbuf[d].reset();
      q.rbuf[d].reset();
    }
    q.cp.reset();
    q.tf.reset();
    q.up.reset();
    q.ld.reset();
    q.p2.reset();
    q.AMP.reset();
    q.CNT.reset();
    q.LINE.reset();
    q.SNAP.reset();
    HIP_OK(hipEventDestroy(q.done));
    HIP_OK(hipEventDestroy(q.copied));
    HIP_OK(hipStreamDestroy(q.st));
    HIP_OK(hipStreamDestroy(q.side));
    q.st = nullptr;
  }
  if (!R.empty()) {
    HIP_OK(hipSetDevice(R[0].dev));
    for (int c = 0; c < 6; ++c) NG[c].reset();
  }
}

template <typename T>
int MultiRun<T>::main() {
  if (const int rc = plan_ranks()) return rc;
  for (int r = 0; r < P; ++r) {
    setup_rank(r);
    if (phys && !setup_physics(r)) return 2;
  }
  enable_peers();
  plan_outputs();
  // --load-from-file: a serial-form checkpoint (either driver's, or a
  // decomposed native run's gathered one) scattered over the ranks
  int t0 = 0;
  if (!s.loadFromFile.empty()) {
    const long got =
        ckpt_load<T>(s, scheme, N, present, [this](int c, const std::vector<T>& host) { scatter(c, host); });
    if (got < 0) return 1;
    t0 = (int)got;
  }
  const int steps = std::max(0, s.numTimeSteps - t0);
  const int warm = std::max(0, std::min(s.warmupSteps, steps));
  run_ckpt(t0, warm);
  sync_all();
  const auto c0 = std::chrono::steady_clock::now();
  ckpt_ms = 0.0;
  run_ckpt(t0 + warm, steps - warm);
  // amplitude mode: after the regular steps, check periods until a step
  // changes no running maximum (native_amp.h)
  const int t_end = amp ? amp_run(t0 + steps) : t0 + steps;
  sync_all();
  HIP_OK(hipGetLastError());
  const double sec =
      std::max(0.0, std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count() - ckpt_ms / 1e3);
  report(sec, t_end, steps, warm);
  return save_results(t_end) ? 0 : 1;
}

template <typename T>
int run_multi(const fdtd::Settings& s) {
  MultiRun<T> m(s);
  return m.main();
}

}  // namespace
