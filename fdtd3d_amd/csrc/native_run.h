// The single-GPU run of the native driver: one state object whose named
// stages are the set-up (fields and coefficients, absorbing layers, the
// chain regions, sources and modes), the pass plans (blocked, hybrid 3D with
// the Drude box, hybrid 2D), the step / pass executors, the run loop
// (warm-up, timed steps, periodic NTFF and checkpoints, amplitude mode) and
// the report -- the counterpart of the reference's single driver
// (Source/main.cpp:36-241 with Scheme3D's init / performSteps) on the same
// kernels and the same plans as the Python driver (models/scheme.py,
// models/blocking.py).
//
// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
#pragma once

#include <memory>

namespace {

template <typename T>
class NativeRun {
 public:
  // plane: 0 = the real run, 1 = the imaginary part of a complex run (the
  // cos / zero source; the update is real-linear, so the two parts step
  // independently -- models/scheme.py planes)
  explicit NativeRun(const fdtd::Settings& s_, int plane_ = 0);
  ~NativeRun();
  // set-up, warm-up, timed steps, report, outputs: the process exit status
  int main();
  // the stages of main (a complex run drives two planes through them)
  bool prepare();
  void run_timed();
  void report_run(double extra_sec = 0.0) const { report(sec_ + extra_sec, t_end_, steps_, warm_); }
  double seconds() const { return sec_; }
  int t_end() const { return t_end_; }
  bool save_complex(const NativeRun<T>& im) const;

 private:
  using ChainFn = int (*)(const void* const*, const double*, const int*, int, int, int, int, void*);

  // ------------------------------------------------------------ configuration
  const fdtd::Settings& s;
  int plane = 0;
  int t0_ = 0, steps_ = 0, warm_ = 0, t_end_ = 0;
  double sec_ = 0.0;
  int dim;
  std::string scheme;
  fdtd::Int3 N;
  std::vector<int> active;
  size_t cells;
  double dx, dt, freq;
  bool vacuum, v4, upml, cpml, tfsf, ntff, amp, use_fused, percell;
  bool cpml_generic = false;
  hipStream_t st = nullptr;

  // ------------------------------------------------- fields and coefficients
  bool present[6];
  Dev<T> F[6], G[6], C[6];
  Dev<float> CE4;  // fp32 3D per-cell: sparse E coefficients of the blocked kernel
  int ebox[6] = {0, 0, 0, 0, 0, 0};
  double cb, db;
  int boxes[36];
  int whole[6];
  int src_comp = 2;
  fdtd::Int3 sp;
  long long src_off = 0;
  bool point_src = true;
  T* Fp[6];

  // ----------------------------------------------------------------- physics
  NativeCpml<T> cpt;
  native_phys::Upml<T> upt;
  Pml2d<T> p2;
  std::vector<IBox> chain_regs, plain_regs;
  std::vector<bool> chain_disp;  // per chain region: holds dispersive cells (the Drude form runs there)
  bool dr_blk = false;
  IBox dr_box = {{0, 0, 0}, {0, 0, 0}};
  ChainFn chain_fn;
  NativeTfsf<T> tft;
  std::unique_ptr<Lowdim2d<T>> ld;
  AmpMode<T> ampm;

  // -------------------------------------------------------------- pass plans
  int T_blk = 1, T2_max = 1, T2_blk = 1;
  bool res1 = false;
  int T_h = 1;
  std::vector<IBox> hcores, hshell[8], hcopy;
  Dev<T> DRS[4], DRL;
  int dr_nid = 0, dr_cur = 0;
  double dr_cbd = 0.0;
  int T2_h = 1;
  std::vector<IBox> h2shell[8], h2copy;
  IBox h2core = {{0, 0, 0}, {0, 0, 0}};
  hipStream_t side[2] = {nullptr, nullptr};
  int nstreams = 3;  // shell streams (--shell-streams; 0 = automatic)
  hipEvent_t fork_ev = nullptr, join_ev[2] = {nullptr, nullptr};
  double ckpt_ms = 0.0;

  // ------------------------------------------------------------------ set-up
  void setup_fields();
  void setup_absorbers();
  void setup_chain_regions();
  void plan_drude();
  bool setup_sources_and_modes();
  void plan_blocking();
  void plan_hybrid3d(int T_h_req);
  void setup_drude_state();
  void plan_hybrid2d();
  void setup_streams();

  // ----------------------------------------------------------- helpers
  double src_val(int t) const;
  void fptrs();
  void clip36(const IBox& r, int* out) const;
  void window_boxes(const IBox& w, int c0, int* out) const;
  void tfsf_kind(int kind);
  void par_windows(const std::vector<IBox>& wins, const std::function<void(const IBox&, hipStream_t)>& fn);
  void par_fns(const std::vector<std::function<void(hipStream_t)>>& fns);

  // ------------------------------------------------------- steps and passes
  void upml_regions(int kind);
  void step(int t);
  void step3d_split(double sv);
  void cpml_slabs(int kind);
  void step2d(double sv);
  void upml_shell(int kind, const std::vector<IBox>& wins);
  void hybrid_pass(int t, int k);
  void hybrid_shell_step(int q, double sv);
  void hybrid2d_pass(int t);
  void blocked2d_pass(int t, int k);
  void blocked3d_pass(int t);
  void advance(int t0, int n);

  // ----------------------------------------------------------------- run loop
  void ntff_report(int t);
  void run_steps(int t0, int n);
  void run_ckpt(int t, int n);
  std::vector<std::pair<void*, size_t>> amp_state();
  void report(double sec, int t_end, int steps, int warm) const;
  bool save_results(int t_end);
};

// ============================================================== configuration

template <typename T>
NativeRun<T>::NativeRun(const fdtd::Settings& s_, int plane_) : s(s_), plane(plane_) {
  dim = s.dimension;
  scheme = dim == 3 ? "3d" : (dim == 2 ? s.mode2D : "1d");
  N = {s.sizeX, dim >= 2 ? s.sizeY : 1, dim == 3 ? s.sizeZ : 1};
  active = dim == 3 ? std::vector<int>{0, 1, 2} : (dim == 2 ? std::vector<int>{0, 1} : std::vector<int>{0});
  cells = (size_t)N[0] * N[1] * N[2];
  dx = s.gridStep;
  dt = dx * s.courantNum / kC;
  freq = kC / s.sourceWaveLength;
  // eps = 1 everywhere (a Drude sphere's eps_inf is 1 too: layout/materials.py Scene.eps)
  vacuum = s.scene == "vacuum" || s.scene == "drude-sphere" || (s.scene == "reference" && dim != 3);
  v4 = sizeof(T) == 4 && N[2] % 4 == 0 && dim == 3;
  // fused / blocked / resident kernels unless --split-kernels (3D fused E+H
  // and blocked passes, 2D blocked passes, 1D one-launch resident run)
  // CPML runs step through the 4-cell-lane split kernels with the psi terms
  // folded in; TF/SF runs apply their corrections between the split half steps
  upml = (s.doUsePML && s.pmlType == "upml") || s.doUseMetamaterials;  // the D/B chain
  cpml = s.doUsePML && !upml;
  tfsf = s.doUseTFSF;
  ntff = s.doUseNTFF && dim == 3;
  // amplitude mode (Scheme3D.cpp:2945-3333): split kernels for the regular
  // steps (the Python driver's choice), then steps with the running maxima
  // until a step changes none; 3D vacuum fp32 folds them into blocked passes
  amp = s.doUseAmplitudeMode;
  use_fused = !s.doUseSplitKernels && !cpml && !tfsf && !upml && !amp;
  percell = !vacuum;
  cb = dt / (kEps0 * dx);
  db = dt / (kMu0 * dx);
  chain_fn = sizeof(T) == 4 ? (ChainFn)fdtd_chain3d_f32 : (ChainFn)fdtd_chain3d_f64;
  HIP_OK(hipStreamCreate(&st));
}

template <typename T>
NativeRun<T>::~NativeRun() {
  for (int q = 0; q < 2; ++q) {
    if (side[q]) HIP_OK(hipStreamDestroy(side[q]));
    if (join_ev[q]) HIP_OK(hipEventDestroy(join_ev[q]));
  }
  if (fork_ev) HIP_OK(hipEventDestroy(fork_ev));
  if (st) HIP_OK(hipStreamDestroy(st));
}

template <typename T>
double NativeRun<T>::src_val(int t) const {
  // (complex runs: the imaginary plane takes the cos / zero source, models/scheme.py source_value)
  if (s.sourceType == "gaussian")
    return plane == 0 ? std::exp(-std::pow((t - s.gaussianDelay) / s.gaussianWidth, 2)) : 0.0;
  return plane == 0 ? std::sin(dt * t * 2 * kPi * freq) : std::cos(dt * t * 2 * kPi * freq);
}

template <typename T>
void NativeRun<T>::fptrs() {
  for (int c = 0; c < 6; ++c) Fp[c] = F[c].p;
}

// ====================================================================== set-up

// field arrays, the per-cell coefficients of a dielectric scene, the update
// boxes of every component and the point source
template <typename T>
void NativeRun<T>::setup_fields() {
  // components present: 0..2 E, 3..5 H
  for (int c = 0; c < 6; ++c) present[c] = dim == 3;
  if (scheme == "tmz") present[2] = present[3] = present[4] = true;
  if (scheme == "tez") present[0] = present[1] = present[5] = true;
  if (scheme == "1d") present[2] = present[4] = true;
  for (int c = 0; c < 6; ++c)
    if (present[c]) {
      F[c].alloc(cells);
      if (use_fused) G[c].alloc(cells);
    }
  if (percell) {
    // per-component averaged eps on the eps layout (2-point E averaging,
    // YeeGridLayout.h:1007-1263); mu = 1 -> constant H arrays
    const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
    auto eps_at = [&](int i, int j, int k) {
      return sphere_eps(i + 0.5, j + 0.5, dim == 3 ? k + 0.5 : ctr[2], ctr, s.sphereRadius, s.sphereEps);
    };
    std::vector<T> host(cells);
    for (int c = 0; c < 6; ++c) {
      if (!present[c]) continue;
      for (int i = 0; i < N[0]; ++i)
        for (int j = 0; j < N[1]; ++j)
          for (int k = 0; k < N[2]; ++k) {
            double v;
            if (c < 3) {
              const int di = c == 0, dj = c == 1 && dim >= 2, dk = c == 2 && dim == 3;
              v = cb * 2.0 / (eps_at(i, j, k) + eps_at(i + di, j + dj, k + dk));
            } else {
              v = db;
            }
            host[((size_t)i * N[1] + j) * N[2] + k] = (T)v;
          }
      C[c].alloc(cells);
      HIP_OK(hipMemcpy(C[c].p, host.data(), cells * sizeof(T), hipMemcpyHostToDevice));
    }
    if (sizeof(T) == 4 && dim == 3) {
      // sparse form for the blocked kernel: the E coefficients of the cells
      // around the sphere (its bounding box + 2 cells; every other cell has
      // eps = 1 on both averaging points, i.e. exactly cb) as one float4 per
      // cell; mu = 1, so H stays on the scalar db
      for (int a = 0; a < 3; ++a) {
        ebox[a] = std::max(0, (int)std::floor(ctr[a] - s.sphereRadius) - 2);
        ebox[3 + a] = std::min(N[a], (int)std::ceil(ctr[a] + s.sphereRadius) + 3);
      }
      const size_t bn = (size_t)std::max(0, ebox[3] - ebox[0]) * std::max(0, ebox[4] - ebox[1]) *
                        std::max(0, ebox[5] - ebox[2]);
      if (bn > 0) {
        std::vector<float> h4(4 * bn, 0.f);
        size_t q = 0;
        for (int i = ebox[0]; i < ebox[3]; ++i)
          for (int j = ebox[1]; j < ebox[4]; ++j)
            for (int k = ebox[2]; k < ebox[5]; ++k, ++q)
              for (int c = 0; c < 3; ++c) {
                const int di = c == 0, dj = c == 1, dk = c == 2;
                h4[4 * q + c] = (float)(cb * 2.0 / (eps_at(i, j, k) + eps_at(i + di, j + dj, k + dk)));
              }
        CE4.alloc(4 * bn);
        HIP_OK(hipMemcpy(CE4.p, h4.data(), 4 * bn * sizeof(float), hipMemcpyHostToDevice));
      }
    }
  }
  for (int c = 0; c < 6; ++c) {
    fdtd::Int3 lo, hi;
    fdtd::global_range(c, N, active, lo, hi);
    for (int a = 0; a < 3; ++a) {
      boxes[6 * c + a] = lo[a];
      boxes[6 * c + 3 + a] = hi[a];
    }
  }
  for (int a = 0; a < 3; ++a) {
    whole[a] = 0;
    whole[3 + a] = N[a];
  }
  // point source (reference Scheme3D.cpp:2011-2022, SchemeTMz.cpp:1345)
  sp = {N[0] / 2, N[1] / 2, N[2] / 2};
  if (scheme == "tmz") sp = {N[0] > 140 ? 70 : N[0] / 2, N[1] / 2, 0};
  if (scheme == "tez") src_comp = 5;
  if (scheme == "1d") sp = {N[0] / 2, 0, 0};
  src_off = ((long long)sp[0] * N[1] + sp[1]) * N[2] + sp[2];
}

// CPML (3D / 2D) and UPML (2D strips, 3D D/B chain with the Drude / Lorentz sphere) tables
template <typename T>
void NativeRun<T>::setup_absorbers() {
  // 3D CPML on rows of a z size not divisible by 4: the scalar split kernels +
  // the generic slab corrections (the 2D form, models/cpml.py)
  cpml_generic = cpml && dim == 3 && N[2] % 4 != 0;
  if (cpml && dim == 3 && !cpml_generic) setup_cpml(cpt, s, N, active, dt, dx);
  if (cpml_generic) setup_cpml2d(p2, s, N, active, present, dt, dx);
  if (dim == 2 && cpml) setup_cpml2d(p2, s, N, active, present, dt, dx);
  if (dim == 2 && upml) {
    // per-cell 1 / (eps eps0) of a dielectric scene (E components; the
    // 2-point averages of the plain coefficients above)
    std::vector<T> inv[3];
    if (percell) {
      const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
      for (int c = 0; c < 3; ++c) {
        if (!present[c]) continue;
        inv[c].resize(cells);
        const int di = c == 0, dj = c == 1;
        for (int i = 0; i < N[0]; ++i)
          for (int j = 0; j < N[1]; ++j) {
            const double a = sphere_eps(i + 0.5, j + 0.5, ctr[2], ctr, s.sphereRadius, s.sphereEps);
            const double b = sphere_eps(i + di + 0.5, j + dj + 0.5, ctr[2], ctr, s.sphereRadius, s.sphereEps);
            inv[c][(size_t)i * N[1] + j] = (T)(1.0 / ((a + b) / 2.0 * kEps0));
          }
      }
    }
    setup_upml2d(p2, s, N, present, dt, dx, inv);
  }
  if (upml && dim == 3) {
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
    native_phys::setup_upml<T>(upt, N, sc, dt, dx);
  }
}

// 3D UPML / Drude: the chain only where it differs from the plain update --
// the PML slabs (one cell of staggering slack) and the dispersive sphere's
// box -- and the plain float4 kernels on the rest (models/scheme.py
// _init_chain_regions; the chain with every sigma and omega zero IS the
// plain update to round-off, and only chain cells read their D levels)
template <typename T>
void NativeRun<T>::setup_chain_regions() {
  if (!(upml && dim == 3)) return;
  const IBox whole_box = {{0, 0, 0}, {N[0], N[1], N[2]}};
  const int pp[3] = {s.doUsePML ? s.pmlSizeX + 1 : 0, s.doUsePML ? s.pmlSizeY + 1 : 0,
                     s.doUsePML ? s.pmlSizeZ + 1 : 0};
  const IBox inner = {{pp[0], pp[1], pp[2]}, {N[0] - pp[0], N[1] - pp[1], N[2] - pp[2]}};
  IBox dbox = {{0, 0, 0}, {0, 0, 0}};
  if (s.doUseMetamaterials) {
    const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
    for (int a = 0; a < 3; ++a) {
      dbox.lo[a] = std::max(0, (int)std::floor(ctr[a] - s.sphereRadius) - 2);
      dbox.hi[a] = std::min(N[a], (int)std::ceil(ctr[a] + s.sphereRadius) + 3);
    }
  }
  bool inside = !inner.empty();
  for (int a = 0; a < 3 && !dbox.empty(); ++a)
    inside = inside && dbox.lo[a] >= inner.lo[a] && dbox.hi[a] <= inner.hi[a];
  if (!inside) {
    chain_regs.push_back(whole_box);
    chain_disp.push_back(true);
  } else {
    if (s.doUsePML) chain_regs = box_minus(whole_box, inner);
    chain_disp.assign(chain_regs.size(), false);
    if (!dbox.empty()) {
      chain_regs.push_back(dbox);
      chain_disp.push_back(true);
      plain_regs = box_minus(inner, dbox);
    } else {
      plain_regs.push_back(inner);
    }
  }
  // region-local D / D1 levels over the chain regions (models/regions.py)
  std::vector<std::array<int, 6>> rb;
  for (const IBox& r : chain_regs) rb.push_back({r.lo[0], r.lo[1], r.lo[2], r.hi[0], r.hi[1], r.hi[2]});
  native_phys::alloc_levels(upt, rb, chain_disp);
}

// Drude box inside the blocked passes (models/blocking.py _plan_drude_blk,
// tb3d_mr.h DrDev, fp64: yee3d_tb64.hip DrDev64): every hybrid pass runs the
// plain blocked core over the box too, then the Drude variant over the box
// grown by T, carrying (delta = D - Dp, Ep) per E component; the stepped
// chain never runs on the box.  3D electric Drude spheres without TF/SF,
// fresh runs (the native checkpoints cover plain media).
template <typename T>
void NativeRun<T>::plan_drude() {
  if (!((v4 || sizeof(T) == 8) && upml && dim == 3 && s.doUseMetamaterials && s.blockedDrude != "off" &&
        s.dispersion != "lorentz" && !tfsf && !amp && !percell && !chain_regs.empty() && !plain_regs.empty() &&
        chain_disp.back() && (upt.disp[0] || upt.disp[1] || upt.disp[2]) && !upt.disp[3] && !upt.disp[4] &&
        !upt.disp[5]))
    return;
  dr_blk = true;
  dr_box = chain_regs.back();
  // the ADE rows must be the Drude form (b1 = -(b0 + b2)) and fit the
  // 8-bit ids: checked HERE, before the hybrid plan keeps the box inside
  // the core -- turning the pass off after planning would leave the box on
  // the plain update (no shell window, no copy box covers it)
  for (int c = 0; c < 3 && dr_blk; ++c) {
    if (!upt.disp[c]) continue;
    if (upt.nlut[c] > 256) dr_blk = false;
    std::vector<T> tab(5 * (size_t)upt.nlut[c]);
    HIP_OK(hipMemcpy(tab.data(), upt.lut[c], tab.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (int q = 0; q < upt.nlut[c]; ++q) {
      const double b0 = tab[5 * q], b1 = tab[5 * q + 1], b2 = tab[5 * q + 2];
      if (std::fabs(b0 + b1 + b2) > 1e-5 * (std::fabs(b0) + std::fabs(b1) + std::fabs(b2))) dr_blk = false;
    }
  }
}

// the TF/SF plane wave, the 2D half-step helper and the amplitude mode's state
template <typename T>
bool NativeRun<T>::setup_sources_and_modes() {
  if (tfsf && !setup_tfsf(tft, s, N, boxes, C, percell ? 1.0 : cb, percell ? 1.0 : db, dt, dx, freq, dim, present))
    return false;
  point_src = !tfsf || s.doUsePointSource;
  // 2D PML half steps and the plain 2D kernels on boxes (native_lowdim.h)
  ld.reset(new Lowdim2d<T>(s, F, C, boxes, N, present, p2, scheme == "tmz", percell, cb, db, st));
  // amplitude mode state (native_amp.h): running maxima, changed counts, the 3D z-line source
  if (amp) ampm.init(s, N, dim == 3 && point_src);
  return true;
}

// steps per pass of the blocked kernels; the hybrid 3D / 2D plans
template <typename T>
void NativeRun<T>::plan_blocking() {
  // --time-block T: T steps per HBM pass through the blocked kernel
  // 0: automatic (5 steps per pass in fp32, 4 in fp64)
  const int T_req = s.timeBlock <= 0 ? (sizeof(T) == 4 ? 5 : 4) : s.timeBlock;
  const int T_max = sizeof(T) == 4 ? fdtd_tb_max_steps() : fdtd_tb64_max_steps();
  T_blk = (scheme == "3d" && use_fused && (v4 || sizeof(T) == 8)) ? std::max(1, std::min(T_max, T_req)) : 1;
  // 2D: yee2d_tb.hip passes (automatic 7 steps), rows of whole 16-byte lanes
  T2_max = sizeof(T) == 4 ? fdtd_tb2d_max_steps() : fdtd_tb2d64_max_steps();
  T2_blk = (dim == 2 && use_fused && N[1] % (16 / (int)sizeof(T)) == 0)
               ? std::max(1, std::min(T2_max, s.timeBlock <= 0 ? 7 : s.timeBlock))
               : 1;
  // 1D: the whole run in one launch of the register-resident kernel
  res1 = dim == 1 && use_fused && N[0] <= fdtd_res1d_max_cells((int)sizeof(T));
  // (fp64: 4 steps per pass, models/blocking.py F64_AUTO_STEPS)
  const int T_h_def = s.hybridBlock == 0 ? (sizeof(T) == 4 ? 5 : 4) : s.hybridBlock;
  if (dr_blk) {
    // (models/blocking.py DRUDE_AUTO_STEPS: the Drude variant holds T - 1 levels in registers)
    const int T_dr = s.hybridBlock > 0 ? s.hybridBlock : (s.timeBlock > 0 ? s.timeBlock : 4);
    if (T_dr > 1 && T_dr <= 5) plan_hybrid3d(T_dr);
    // the Drude pass runs inside hybrid passes only; when it does not fit, the
    // stepped dispersive box cut out of the core at the usual hybrid T
    if (T_dr <= 1 || T_dr > 5 || !dr_blk || T_h <= 1) {
      dr_blk = false;
      T_h = 1;
    }
  }
  if (!dr_blk) plan_hybrid3d(T_h_def);
  if (dr_blk) setup_drude_state();
  plan_hybrid2d();
}

// Hybrid passes for 3D fp32 CPML / UPML / Drude / TF/SF runs -- the plan the
// Python driver picks automatically (models/blocking.py _hybrid_plan): every
// T steps the blocked kernel advances the core (cells at least T + 2 beyond
// every absorbing slab, TF/SF target and stepped dispersive box) by T steps
// F -> G; the shell is stepped in place in F with a band T - s deep into the
// core at step s (stale core values corrupt one band cell per step, so the
// shell itself stays exact), copied into G, and the buffers swap.
template <typename T>
void NativeRun<T>::plan_hybrid3d(int T_h_req) {
  // (UPML runs without dispersive media too: the chain slabs run whole in
  // every shell step, the plain kernels on the windows' inner parts)
  const bool upml_h = upml && s.doUsePML && !s.doUseMetamaterials && plain_regs.size() == 1;
  // Drude / Lorentz sphere (+ UPML): the dispersive box is cut out of the core
  // (grown by T + 2) and stepped with the shell, chain whole every step
  IBox dbox_h = {{0, 0, 0}, {0, 0, 0}};
  if (upml && s.doUseMetamaterials && !chain_regs.empty() && !plain_regs.empty()) dbox_h = chain_regs.back();
  const bool drude_h = !dbox_h.empty();
  // TF/SF without absorbing layers: the shell is the TF/SF band on the plain kernels
  const bool tfsf_h = tfsf && !s.doUsePML && !upml;
  // (fp32 rows of float4 lanes; fp64: the CPML windows' 4-cell double groups)
  const bool rows_ok = sizeof(T) == 4 ? v4 : N[2] % 4 == 0;
  const int tb_max = sizeof(T) == 4 ? fdtd_tb_max_steps() : fdtd_tb64_max_steps();
  if (!(scheme == "3d" && rows_ok && (cpml || upml_h || drude_h || tfsf_h) && !percell && !amp && T_h_req > 1 &&
        T_h_req <= tb_max))
    return;
  const int Th = T_h_req;
  const int pml[3] = {s.doUsePML ? s.pmlSizeX + (upml ? 1 : 0) : 0, s.doUsePML ? s.pmlSizeY + (upml ? 1 : 0) : 0,
                      s.doUsePML ? s.pmlSizeZ + (upml ? 1 : 0) : 0};
  const int tfs[3] = {s.tfsfSizeX, s.tfsfSizeY, s.tfsfSizeZ};
  const IBox alloc = {{0, 0, 0}, {N[0], N[1], N[2]}};
  IBox K;
  for (int a = 0; a < 3; ++a) {
    const int edge = std::max(pml[a], tfsf ? tfs[a] + 1 : 0);
    // nothing irregular along an axis but the domain border: the core
    // reaches the faces (the blocked kernel handles them itself)
    K.lo[a] = edge > 0 ? edge + Th + 2 : 0;
    K.hi[a] = edge > 0 ? N[a] - edge - Th - 2 : N[a];
  }
  auto grow = [&](const IBox& b, int n) {
    IBox g = b;
    for (int a = 0; a < 3; ++a) {
      g.lo[a] -= n;
      g.hi[a] += n;
    }
    return g;
  };
  auto shrink_inner = [&](const IBox& b, int n) {
    IBox r = b;
    for (int a = 0; a < 3; ++a) {
      if (r.lo[a] > 0) r.lo[a] += n;
      if (r.hi[a] < N[a]) r.hi[a] -= n;
    }
    return r;
  };
  IBox Dm = {{0, 0, 0}, {0, 0, 0}};
  bool ok = !K.empty();
  if (ok && dr_blk) {
    // the Drude pass's output (the box grown by T, clipped to the grid) inside the core
    const IBox g = box_and(grow(dr_box, Th), alloc);
    for (int a = 0; a < 3; ++a) dr_blk = dr_blk && g.lo[a] >= K.lo[a] && g.hi[a] <= K.hi[a];
  }
  if (ok && drude_h && !dr_blk) {
    Dm = box_and(grow(dbox_h, Th + 2), K);
    // the dispersive box runs whole in every shell step: inside every window set
    const IBox KT = shrink_inner(K, Th);
    for (int a = 0; a < 3; ++a) ok = ok && dbox_h.lo[a] >= KT.lo[a] && dbox_h.hi[a] <= KT.hi[a];
  }
  std::vector<IBox> cores;
  if (ok) cores = Dm.empty() ? std::vector<IBox>{K} : box_minus(K, Dm);
  long long vol = 0;
  for (const IBox& b : cores) vol += b.volume();
  if (!(ok && vol >= (long long)cells / 4)) return;
  // the shell windows of every step and the copy boxes: the one geometry the
  // Python driver plans too (host_native.cpp fdtd::hybrid_windows)
  auto b6 = [](const IBox& b) { return fdtd::Box6{b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2]}; };
  auto ib = [](const fdtd::Box6& b) { return IBox{{b[0], b[1], b[2]}, {b[3], b[4], b[5]}}; };
  const bool act[3] = {true, true, true};
  std::vector<std::vector<fdtd::Box6>> shells;
  std::vector<fdtd::Box6> copy;
  if (!fdtd::hybrid_windows(b6(alloc), b6(K), b6(Dm), Th, act, N, shells, copy)) return;
  T_h = Th;
  hcores = cores;
  for (int q = 0; q < T_h; ++q) {
    hshell[q].clear();
    for (const auto& w : shells[q]) hshell[q].push_back(ib(w));
  }
  hcopy.clear();
  for (const auto& w : copy) hcopy.push_back(ib(w));
  for (int c = 0; c < 6; ++c)
    if (present[c] && !G[c].p) G[c].alloc(cells);
}

// the Drude pass's state (two sets of two float4 arrays over the box; the
// material ids of Ex | Ey << 8 | Ez << 16 in .w of the first) and its
// (b0 cbd, b2, m1, m2) rows per component
template <typename T>
void NativeRun<T>::setup_drude_state() {
  const int bn[3] = {dr_box.hi[0] - dr_box.lo[0], dr_box.hi[1] - dr_box.lo[1], dr_box.hi[2] - dr_box.lo[2]};
  const size_t nb = (size_t)bn[0] * bn[1] * bn[2];
  const double two = 2 * kEps0;
  dr_cbd = (double)(T)((two * dt / dx) / two);  // the chain's cbD where sigma = 0
  std::vector<unsigned> ids(nb, 0u);
  for (int c = 0; c < 3; ++c) {
    if (upt.disp[c]) {
      dr_nid = std::max(dr_nid, upt.nlut[c]);
      std::vector<unsigned char> full(cells);
      HIP_OK(hipMemcpy(full.data(), upt.ids[c], cells, hipMemcpyDeviceToHost));
      for (int i = 0; i < bn[0]; ++i)
        for (int j = 0; j < bn[1]; ++j)
          for (int k = 0; k < bn[2]; ++k)
            ids[((size_t)i * bn[1] + j) * bn[2] + k] |=
                (unsigned)full[((size_t)(i + dr_box.lo[0]) * N[1] + j + dr_box.lo[1]) * N[2] + k + dr_box.lo[2]]
                << (8 * c);
    } else {
      dr_nid = std::max(dr_nid, 1);  // id 0: the plain row (cb, 0, 1, 0)
    }
  }
  if (dr_nid > 256) {  // excluded before the hybrid plan (plan_drude)
    std::fprintf(stderr, "internal error: Drude LUT of %d rows after planning\n", dr_nid);
    std::exit(3);
  }
  std::vector<T> rows((size_t)3 * dr_nid * 4, T(0));
  for (int c = 0; c < 3; ++c) {
    T* r = rows.data() + (size_t)c * dr_nid * 4;
    if (!upt.disp[c]) {
      r[0] = (T)cb;
      r[2] = T(1);
      continue;
    }
    std::vector<T> tab(5 * (size_t)upt.nlut[c]);
    HIP_OK(hipMemcpy(tab.data(), upt.lut[c], tab.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (int q = 0; q < upt.nlut[c]; ++q) {
      r[4 * q] = (T)((double)tab[5 * q] * dr_cbd);
      r[4 * q + 1] = tab[5 * q + 2];
      r[4 * q + 2] = tab[5 * q + 3];
      r[4 * q + 3] = tab[5 * q + 4];
    }
  }
  DRL.alloc(rows.size());
  HIP_OK(hipMemcpy(DRL.p, rows.data(), rows.size() * sizeof(T), hipMemcpyHostToDevice));
  // the ids' bits in the first 4 bytes of the fourth element (fp64: its low word)
  std::vector<T> s0(4 * nb, T(0));
  for (size_t e = 0; e < nb; ++e) std::memcpy(&s0[4 * e + 3], &ids[e], 4);
  for (int q = 0; q < 4; ++q) DRS[q].alloc(4 * nb);
  HIP_OK(hipMemcpy(DRS[0].p, s0.data(), s0.size() * sizeof(T), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(DRS[2].p, s0.data(), s0.size() * sizeof(T), hipMemcpyHostToDevice));
}

// 2D hybrid passes (models/blocking.py on yee2d_tb.hip): every T steps the
// 2D blocked kernel advances the core (cells at least T + 2 beyond the
// absorbing strips and the TF/SF targets) F -> G; the shell strips step in
// place in F with a band T - s deep into the core at step s (absorbing
// strips whole), are copied into G, and the buffers swap
template <typename T>
void NativeRun<T>::plan_hybrid2d() {
  if (!(dim == 2 && (cpml || (upml && !s.doUseMetamaterials)) && !percell && !amp && !s.doUseSplitKernels &&
        N[1] % (16 / (int)sizeof(T)) == 0))
    return;
  const int Th = s.hybridBlock == 0 ? 7 : s.hybridBlock;
  if (!(Th > 1 && Th <= T2_max)) return;
  const int pml[2] = {s.pmlSizeX + (upml ? 1 : 0), s.pmlSizeY + (upml ? 1 : 0)};
  const int tfs[2] = {s.tfsfSizeX, s.tfsfSizeY};
  IBox K = {{0, 0, 0}, {N[0], N[1], 1}};
  for (int a = 0; a < 2; ++a) {
    const int edge = std::max(pml[a], tfsf ? tfs[a] + 1 : 0);
    K.lo[a] = edge + Th + 2;
    K.hi[a] = N[a] - edge - Th - 2;
  }
  if (K.empty() || K.volume() < (long long)cells / 4) return;
  T2_h = Th;
  h2core = K;
  const IBox alloc = {{0, 0, 0}, {N[0], N[1], 1}};
  for (int q = 0; q < T2_h; ++q) {
    IBox Kd = K;
    for (int a = 0; a < 2; ++a) {
      Kd.lo[a] += T2_h - q;
      Kd.hi[a] -= T2_h - q;
    }
    for (const IBox& w : box_minus(alloc, Kd))
      if (!w.empty()) h2shell[q].push_back(w);
  }
  for (const IBox& b : box_minus(alloc, K))
    if (!b.empty()) h2copy.push_back(b);
  for (int c = 0; c < 6; ++c)
    if (present[c] && !G[c].p) G[c].alloc(cells);
}

// independent shell-window launches of a half step side by side on three
// streams (the tail of one small launch overlaps the next; models/scheme.py
// _par_launches), joined back into `st`
template <typename T>
void NativeRun<T>::setup_streams() {
  if (T_h <= 1) return;
  nstreams = s.shellStreams > 0 ? std::min(3, s.shellStreams) : 3;
  for (int q = 0; q < 2; ++q) {
    HIP_OK(hipStreamCreateWithFlags(&side[q], hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&join_ev[q], hipEventDisableTiming));
  }
  HIP_OK(hipEventCreateWithFlags(&fork_ev, hipEventDisableTiming));
}

// ===================================================================== helpers

template <typename T>
void NativeRun<T>::clip36(const IBox& r, int* out) const {
  for (int c = 0; c < 6; ++c) {
    IBox b;
    for (int a = 0; a < 3; ++a) {
      b.lo[a] = boxes[6 * c + a];
      b.hi[a] = boxes[6 * c + 3 + a];
    }
    b = box_and(b, r);
    for (int a = 0; a < 3; ++a) {
      out[6 * c + a] = b.empty() ? 0 : b.lo[a];
      out[6 * c + 3 + a] = b.empty() ? 0 : b.hi[a];
    }
  }
}

template <typename T>
void NativeRun<T>::window_boxes(const IBox& w, int c0, int* out) const {
  for (int c = c0; c < c0 + 3; ++c) {
    IBox b;
    for (int a = 0; a < 3; ++a) {
      b.lo[a] = boxes[6 * c + a];
      b.hi[a] = boxes[6 * c + 3 + a];
    }
    b = box_and(b, w);
    for (int a = 0; a < 3; ++a) {
      out[6 * (c - c0) + a] = b.empty() ? 0 : b.lo[a];
      out[6 * (c - c0) + 3 + a] = b.empty() ? 0 : b.hi[a];
    }
  }
}

template <typename T>
void NativeRun<T>::tfsf_kind(int kind) {
  for (int c = 3 * kind; c < 3 * kind + 3; ++c)
    for (auto* l : tft.tab[c]) K_OK(tfsf_apply(F[c].p, *l, kind == 0 ? tft.hinc.p : tft.einc.p, whole, st));
}

template <typename T>
void NativeRun<T>::par_windows(const std::vector<IBox>& wins,
                               const std::function<void(const IBox&, hipStream_t)>& fn) {
  if (wins.size() <= 1 || !side[0]) {
    for (const IBox& w : wins) fn(w, st);
    return;
  }
  const int ns = nstreams;
  HIP_OK(hipEventRecord(fork_ev, st));
  for (int q = 0; q < ns - 1; ++q) HIP_OK(hipStreamWaitEvent(side[q], fork_ev, 0));
  for (size_t n = 0; n < wins.size(); ++n) fn(wins[n], n % ns == 0 ? st : side[n % ns - 1]);
  for (int q = 0; q < ns - 1; ++q) {
    HIP_OK(hipEventRecord(join_ev[q], side[q]));
    HIP_OK(hipStreamWaitEvent(st, join_ev[q], 0));
  }
}

// independent launches of a half step (disjoint cells) round-robin on the
// three streams, joined back into `st` (models/scheme.py _par_launches)
template <typename T>
void NativeRun<T>::par_fns(const std::vector<std::function<void(hipStream_t)>>& fns) {
  if (fns.size() <= 1 || !side[0]) {
    for (const auto& fn : fns) fn(st);
    return;
  }
  const int ns = nstreams;
  HIP_OK(hipEventRecord(fork_ev, st));
  for (int q = 0; q < ns - 1; ++q) HIP_OK(hipStreamWaitEvent(side[q], fork_ev, 0));
  for (size_t n = 0; n < fns.size(); ++n) fns[n](n % ns == 0 ? st : side[n % ns - 1]);
  for (int q = 0; q < ns - 1; ++q) {
    HIP_OK(hipEventRecord(join_ev[q], side[q]));
    HIP_OK(hipStreamWaitEvent(st, join_ev[q], 0));
  }
}

// =========================================================== steps and passes

template <typename T>
void NativeRun<T>::upml_regions(int kind) {
  fptrs();
  int rb[36];
  for (size_t q = 0; q < chain_regs.size(); ++q) {
    clip36(chain_regs[q], rb);
    K_OK(native_phys::upml_kind<T>(upt, Fp, rb, kind, N[1], N[2], st, chain_fn, false, !chain_disp[q], nullptr, 1.0,
                                   (int)q));
  }
  native_phys::upml_rotate(upt, kind);
  for (const IBox& r : plain_regs) {
    clip36(r, rb);
    if (kind == 0)
      K_OK(e3d(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p, percell ? 1.0 : cb, N[0],
               N[1], N[2], rb, 0, st, v4));
    else
      K_OK(h3d(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p, percell ? 1.0 : db, N[0],
               N[1], N[2], rb + 18, 0, st, v4));
  }
}

// one time step (t) through the configured kernels
template <typename T>
void NativeRun<T>::step(int t) {
  const double sv = src_val(t);
  if (scheme == "3d") {
    if (use_fused) {
      const T* ei[3] = {F[0].p, F[1].p, F[2].p};
      const T* hi[3] = {F[3].p, F[4].p, F[5].p};
      T* eo[3] = {G[0].p, G[1].p, G[2].p};
      T* ho[3] = {G[3].p, G[4].p, G[5].p};
      const T* cbs[3] = {C[0].p, C[1].p, C[2].p};
      const T* dbs[3] = {C[3].p, C[4].p, C[5].p};
      K_OK(fused(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], N[1], N[2], boxes, src_off,
                 src_comp, sv, st, v4));
      for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
    } else {
      step3d_split(sv);
    }
  } else if (scheme == "tmz" || scheme == "tez") {
    step2d(sv);
  } else {
    K_OK(e1d(F[2].p, F[4].p, C[2].p, percell ? 1.0 : cb, boxes[12], boxes[15], st));
    K_OK(setv(F[2].p, src_off, sv, st));
    K_OK(h1d(F[4].p, F[2].p, C[4].p, percell ? 1.0 : db, boxes[24], boxes[27], st));
  }
}

// split half steps: [incident line E] E update [TF/SF on E] [source]
// [incident line H] H update [TF/SF on H] -- the order of scheme.step
template <typename T>
void NativeRun<T>::step3d_split(double sv) {
  if (tfsf) K_OK(inc_e(tft.einc.p, tft.hinc.p, tft.nline, tft.ce, sv, st));
  if (upml) {
    upml_regions(0);
  } else if (cpml_generic) {
    K_OK(e3d(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p, percell ? 1.0 : cb, N[0], N[1],
             N[2], boxes, 0, st, false));
    cpml_slabs(0);
  } else if (cpml) {
    // (4-cell z lanes: float4 / double4)
    if constexpr (sizeof(T) == 4)
      K_OK(fdtd_update_e3d_cpml_v4_f32(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p,
                                       percell ? 1.0 : cb, N[0], N[1], N[2], boxes, 0, cpt.P[0].data(),
                                       cpt.I[0].data(), st));
    else
      K_OK(fdtd_update_e3d_cpml_v4_f64(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p,
                                       percell ? 1.0 : cb, N[0], N[1], N[2], boxes, 0, cpt.P[0].data(),
                                       cpt.I[0].data(), st));
  } else {
    K_OK(e3d(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p, percell ? 1.0 : cb, N[0], N[1],
             N[2], boxes, 0, st, v4));
  }
  if (tfsf) tfsf_kind(0);
  if (point_src) {
    if (ampm.active && ampm.line_n > 0)  // the amplitude mode's Ez z-line replaces the point source
      K_OK(setvs(F[2].p, ampm.LINE.p, ampm.line_n, sv, st));
    else
      K_OK(setv(F[src_comp].p, src_off, sv, st));
  }
  if (tfsf) K_OK(inc_h(tft.einc.p, tft.hinc.p, tft.nline, tft.ch, st));
  if (upml) {
    upml_regions(1);
  } else if (cpml_generic) {
    K_OK(h3d(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p, percell ? 1.0 : db, N[0], N[1],
             N[2], boxes + 18, 0, st, false));
    cpml_slabs(1);
  } else if (cpml) {
    if constexpr (sizeof(T) == 4)
      K_OK(fdtd_update_h3d_cpml_v4_f32(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p,
                                       percell ? 1.0 : db, N[0], N[1], N[2], boxes + 18, 0, cpt.P[1].data(),
                                       cpt.I[1].data(), st));
    else
      K_OK(fdtd_update_h3d_cpml_v4_f64(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p,
                                       percell ? 1.0 : db, N[0], N[1], N[2], boxes + 18, 0, cpt.P[1].data(),
                                       cpt.I[1].data(), st));
  } else {
    K_OK(h3d(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p, percell ? 1.0 : db, N[0], N[1],
             N[2], boxes + 18, 0, st, v4));
  }
  if (tfsf) tfsf_kind(1);
}

// the generic CPML slab corrections of one kind (0 = E) after the plain
// update (3D rows of a z size not divisible by 4; native_lowdim.h cpml)
template <typename T>
void NativeRun<T>::cpml_slabs(int kind) {
  for (const Slab2d<T>& sl : p2.slabs) {
    if ((sl.comp < 3) != (kind == 0)) continue;
    const void* cp[4] = {nullptr, nullptr, nullptr, percell ? (const void*)C[sl.comp].p : nullptr};
    K_OK(cpml_apply(F[sl.comp].p, F[sl.src].p, sl.psi, sl.axis, sl.sign, kind == 0 ? 1 : 0, sl.b, sl.c, sl.k,
                    percell ? 1.0 : (kind == 0 ? cb : db), cp, N[1], N[2], sl.box, sl.pbox, st));
  }
}

// [incident line E] E update (+ CPML slabs | UPML chain) [TF/SF on E]
// [source] [incident line H] H update [TF/SF on H]
template <typename T>
void NativeRun<T>::step2d(double sv) {
  const bool tm = scheme == "tmz";
  if (tfsf) K_OK(inc_e(tft.einc.p, tft.hinc.p, tft.nline, tft.ce, sv, st));
  if (upml)
    ld->upml(0);
  else if (tm)
    K_OK(tmz_e(F[2].p, F[3].p, F[4].p, C[2].p, percell ? 1.0 : cb, N[0], N[1], boxes + 12, st));
  else
    K_OK(tez_e(F[0].p, F[1].p, F[5].p, C[0].p, C[1].p, percell ? 1.0 : cb, N[0], N[1], boxes, st));
  if (cpml) ld->cpml(0);
  if (tfsf) tfsf_kind(0);
  if (point_src) K_OK(setv(F[src_comp].p, src_off, sv, st));  // hard source between the E and H updates
  if (tfsf) K_OK(inc_h(tft.einc.p, tft.hinc.p, tft.nline, tft.ch, st));
  if (upml) {
    ld->upml(1);
  } else if (tm) {
    int hb[12];
    std::memcpy(hb, boxes + 18, 12 * sizeof(int));
    K_OK(tmz_h(F[3].p, F[4].p, F[2].p, C[3].p, C[4].p, percell ? 1.0 : db, N[0], N[1], hb, st));
  } else {
    K_OK(tez_h(F[5].p, F[0].p, F[1].p, C[5].p, percell ? 1.0 : db, N[0], N[1], boxes + 30, st));
  }
  if (cpml) ld->cpml(1);
  if (tfsf) tfsf_kind(1);
}

// UPML shell half step: the chain slabs whole (they lie inside every
// step's windows), the plain kernels on the windows' parts in the inner box
// (chain slabs and plain window parts are disjoint: side by side on the
// three streams, as the Python driver's shell -- the float4 plain kernels
// store only their own elements of a 4-cell group that straddles an
// unaligned z border with a chain box; the level rotation is a host pointer
// swap after the launches captured their pointers)
// A thin plain part on the z side of a non-dispersive chain slab with a
// footprint inside the slab's rides in that slab's chain launch (its rows
// are read once, whole; models/scheme.py _chain_plan "fold").
template <typename T>
void NativeRun<T>::upml_shell(int kind, const std::vector<IBox>& wins) {
  fptrs();
  std::vector<std::function<void(hipStream_t)>> fns, pfns;
  std::vector<IBox> parts;
  for (const IBox& w : wins)
    for (const IBox& pr : plain_regs) {
      const IBox b = box_and(w, pr);
      if (!b.empty()) parts.push_back(b);
    }
  std::vector<int> fold(chain_regs.size(), -1);
  std::vector<bool> folded(parts.size(), false);
  for (size_t n = 0; n < parts.size(); ++n) {
    const IBox& b = parts[n];
    if (b.hi[2] - b.lo[2] > 64) continue;
    for (size_t q = 0; q < chain_regs.size(); ++q) {
      const IBox& cr = chain_regs[q];
      if (fold[q] >= 0 || chain_disp[q] || (dr_blk && q + 1 == chain_regs.size())) continue;
      if (b.lo[0] < cr.lo[0] || b.hi[0] > cr.hi[0] || b.lo[1] < cr.lo[1] || b.hi[1] > cr.hi[1]) continue;
      if (b.lo[2] != cr.hi[2] && b.hi[2] != cr.lo[2]) continue;
      fold[q] = (int)n;
      folded[n] = true;
      break;
    }
  }
  for (size_t q = 0; q < chain_regs.size(); ++q) {
    if (dr_blk && q + 1 == chain_regs.size()) continue;  // the Drude box: inside the blocked passes
    fns.push_back([&, q, kind](hipStream_t ss) {
      int rb[36], pb[36];
      clip36(chain_regs[q], rb);
      if (fold[q] >= 0) clip36(parts[fold[q]], pb);
      K_OK(native_phys::upml_kind<T>(upt, Fp, rb, kind, N[1], N[2], ss, chain_fn, false, !chain_disp[q],
                                     fold[q] >= 0 ? pb : nullptr, kind == 0 ? cb : db, (int)q));
    });
  }
  for (size_t n = 0; n < parts.size(); ++n) {
    if (folded[n]) continue;
    const IBox b = parts[n];
    pfns.push_back([&, b, kind](hipStream_t ss) {
      int rb[36];
      clip36(b, rb);
      if (kind == 0)
        K_OK(e3d(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p, cb, N[0], N[1], N[2], rb, 0,
                 ss, v4));
      else
        K_OK(h3d(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p, db, N[0], N[1], N[2],
                 rb + 18, 0, ss, v4));
    });
  }
  fns.insert(fns.end(), pfns.begin(), pfns.end());
  par_fns(fns);
  native_phys::upml_rotate(upt, kind);
}

// one pass of k <= T_h steps (a shorter pass steps the shell windows of the
// pass's last k steps: band depth k - q at step q)
template <typename T>
void NativeRun<T>::hybrid_pass(int t, int k) {
  {
    const T* ei[3] = {F[0].p, F[1].p, F[2].p};
    const T* hi[3] = {F[3].p, F[4].p, F[5].p};
    T* eo[3] = {G[0].p, G[1].p, G[2].p};
    T* ho[3] = {G[3].p, G[4].p, G[5].p};
    const T* none3[3] = {nullptr, nullptr, nullptr};
    double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int l = 0; l < k; ++l) vals[l] = src_val(t + l);
    for (const IBox& hc : hcores) {
      bool in_core = true;
      for (int a = 0; a < 3; ++a) in_core = in_core && sp[a] >= hc.lo[a] && sp[a] < hc.hi[a];
      const int src[4] = {sp[0], sp[1], sp[2], point_src && in_core ? src_comp : -1};
      const int ob[6] = {hc.lo[0], hc.lo[1], hc.lo[2], hc.hi[0], hc.hi[1], hc.hi[2]};
      K_OK(tb3d(ei, hi, eo, ho, none3, none3, cb, db, N[0], N[1], N[2], boxes, k, src, vals, st, nullptr, nullptr,
                ob));
    }
    if (dr_blk) {
      // the Drude pass over the box grown by k (overwrites the core pass there)
      int ob[6], bb[6];
      for (int a = 0; a < 3; ++a) {
        ob[a] = std::max(0, dr_box.lo[a] - k);
        ob[3 + a] = std::min(N[a], dr_box.hi[a] + k);
        bb[a] = dr_box.lo[a];
        bb[3 + a] = dr_box.hi[a];
      }
      const int src[4] = {sp[0], sp[1], sp[2], point_src ? src_comp : -1};
      void* sin[2] = {DRS[2 * dr_cur].p, DRS[2 * dr_cur + 1].p};
      void* sout[2] = {DRS[2 * (1 - dr_cur)].p, DRS[2 * (1 - dr_cur) + 1].p};
      K_OK(drude3d(ei, hi, eo, ho, cb, db, N[0], N[1], N[2], boxes, ob, k, src, vals, bb, sin, sout, DRL.p, dr_nid,
                   dr_cbd, st));
      dr_cur ^= 1;
    }
    for (int q0 = 0; q0 < k; ++q0) hybrid_shell_step(T_h - k + q0, src_val(t + q0));  // band depth k - q0
    T* src6[6] = {F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p};
    T* dst6[6] = {G[0].p, G[1].p, G[2].p, G[3].p, G[4].p, G[5].p};
    for (const IBox& b : hcopy) {
      const int bx[6] = {b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2]};
      K_OK(xfer(src6, dst6, 6, N[1], N[2], bx, st));
    }
    for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
  }
}

// one stepped step of the hybrid shell on window set q, in place in F
template <typename T>
void NativeRun<T>::hybrid_shell_step(int q, double sv) {
  {
    T* const F6[6] = {F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p};
    const T* const none6[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (tfsf) K_OK(inc_e(tft.einc.p, tft.hinc.p, tft.nline, tft.ce, sv, st));
    if (upml) {
      upml_shell(0, hshell[q]);
    } else if (!cpml) {
      par_windows(hshell[q], [&](const IBox& w, hipStream_t ss) {
        int rb[36];
        clip36(w, rb);
        K_OK(e3d(F[0].p, F[1].p, F[2].p, F[3].p, F[4].p, F[5].p, C[0].p, C[1].p, C[2].p, cb, N[0], N[1], N[2], rb, 0,
                 ss, v4));
      });
    } else {
      par_windows(hshell[q], [&](const IBox& w, hipStream_t ss) {
        int wb2[18];
        window_boxes(w, 0, wb2);
        K_OK(cpml_e3d(F6, none6, cb, N[0], N[1], N[2], wb2, cpt.P[0].data(), cpt.I[0].data(), ss));
      });
    }
    if (tfsf) tfsf_kind(0);
    if (point_src) K_OK(setv(F[src_comp].p, src_off, sv, st));
    if (tfsf) K_OK(inc_h(tft.einc.p, tft.hinc.p, tft.nline, tft.ch, st));
    if (upml) {
      upml_shell(1, hshell[q]);
    } else if (!cpml) {
      par_windows(hshell[q], [&](const IBox& w, hipStream_t ss) {
        int rb[36];
        clip36(w, rb);
        K_OK(h3d(F[3].p, F[4].p, F[5].p, F[0].p, F[1].p, F[2].p, C[3].p, C[4].p, C[5].p, db, N[0], N[1], N[2],
                 rb + 18, 0, ss, v4));
      });
    } else {
      par_windows(hshell[q], [&](const IBox& w, hipStream_t ss) {
        int wb2[18];
        window_boxes(w, 3, wb2);
        K_OK(cpml_h3d(F6, none6, db, N[0], N[1], N[2], wb2, cpt.P[1].data(), cpt.I[1].data(), ss));
      });
    }
    if (tfsf) tfsf_kind(1);
  }
}

template <typename T>
void NativeRun<T>::hybrid2d_pass(int t) {
  const int ord[2][3] = {{2, 3, 4}, {0, 1, 5}};  // TMz Ez Hx Hy, TEz Ex Ey Hz
  const int m = scheme == "tmz" ? 0 : 1;
  const int* o = ord[m];
  const T* ei[2] = {F[o[0]].p, m ? F[o[1]].p : nullptr};
  const T* hi[2] = {F[m ? o[2] : o[1]].p, m ? nullptr : F[o[2]].p};
  T* eo[2] = {G[o[0]].p, m ? G[o[1]].p : nullptr};
  T* ho[2] = {G[m ? o[2] : o[1]].p, m ? nullptr : G[o[2]].p};
  const T* cs[3] = {C[o[0]].p, C[o[1]].p, C[o[2]].p};
  int b2[18];
  for (int q = 0; q < 3; ++q) std::memcpy(b2 + 6 * q, boxes + 6 * o[q], 6 * sizeof(int));
  const int ob[6] = {h2core.lo[0], h2core.lo[1], 0, h2core.hi[0], h2core.hi[1], 1};
  const bool in_core = sp[0] >= h2core.lo[0] && sp[0] < h2core.hi[0] && sp[1] >= h2core.lo[1] && sp[1] < h2core.hi[1];
  const int src[3] = {sp[0], sp[1], point_src && in_core ? (m ? 2 : 0) : -1};
  double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int l = 0; l < T2_h; ++l) vals[l] = src_val(t + l);
  K_OK(tb2d(m, ei, hi, eo, ho, cs, cb, db, N[0], N[1], b2, ob, T2_h, src, vals, st));
  const IBox& inner2 = ld->inner;
  for (int q = 0; q < T2_h; ++q) {
    const double sv = src_val(t + q);
    if (tfsf) K_OK(inc_e(tft.einc.p, tft.hinc.p, tft.nline, tft.ce, sv, st));
    if (upml) {
      ld->upml_chain(0);
      for (const IBox& w : h2shell[q]) ld->plain(0, box_and(w, inner2));
    } else {
      for (const IBox& w : h2shell[q]) ld->plain(0, w);
      ld->cpml(0);
    }
    if (tfsf) tfsf_kind(0);
    if (point_src) K_OK(setv(F[src_comp].p, src_off, sv, st));
    if (tfsf) K_OK(inc_h(tft.einc.p, tft.hinc.p, tft.nline, tft.ch, st));
    if (upml) {
      ld->upml_chain(1);
      for (const IBox& w : h2shell[q]) ld->plain(1, box_and(w, inner2));
    } else {
      for (const IBox& w : h2shell[q]) ld->plain(1, w);
      ld->cpml(1);
    }
    if (tfsf) tfsf_kind(1);
  }
  T* src3[3] = {F[o[0]].p, F[o[1]].p, F[o[2]].p};
  T* dst3[3] = {G[o[0]].p, G[o[1]].p, G[o[2]].p};
  for (const IBox& b : h2copy) {
    const int bx[6] = {b.lo[0], b.lo[1], b.lo[2], b.hi[0], b.hi[1], b.hi[2]};
    K_OK(xfer(src3, dst3, 3, N[1], N[2], bx, st));
  }
  for (int q = 0; q < 3; ++q) std::swap(F[o[q]].p, G[o[q]].p);
}

// k <= T2_blk steps of the whole 2D grid in one blocked pass
template <typename T>
void NativeRun<T>::blocked2d_pass(int t, int k) {
  // component order: TMz Ez Hx Hy, TEz Ex Ey Hz
  const int ord[2][3] = {{2, 3, 4}, {0, 1, 5}};
  const int m = scheme == "tmz" ? 0 : 1;
  const int* o = ord[m];
  const T* ei[2] = {F[o[0]].p, m ? F[o[1]].p : nullptr};
  const T* hi[2] = {F[m ? o[2] : o[1]].p, m ? nullptr : F[o[2]].p};
  T* eo[2] = {G[o[0]].p, m ? G[o[1]].p : nullptr};
  T* ho[2] = {G[m ? o[2] : o[1]].p, m ? nullptr : G[o[2]].p};
  const T* cs[3] = {C[o[0]].p, C[o[1]].p, C[o[2]].p};
  int b2[18];
  for (int q = 0; q < 3; ++q) std::memcpy(b2 + 6 * q, boxes + 6 * o[q], 6 * sizeof(int));
  const int ob[6] = {0, 0, 0, N[0], N[1], 1};
  const int src[3] = {sp[0], sp[1], m ? 2 : 0};
  double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int l = 0; l < k; ++l) vals[l] = src_val(t + l);
  K_OK(tb2d(m, ei, hi, eo, ho, cs, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], N[1], b2, ob, k, src, vals, st));
  for (int q = 0; q < 3; ++q) std::swap(F[o[q]].p, G[o[q]].p);
}

// T_blk steps of the whole 3D grid in one blocked pass
template <typename T>
void NativeRun<T>::blocked3d_pass(int t) {
  const T* ei[3] = {F[0].p, F[1].p, F[2].p};
  const T* hi[3] = {F[3].p, F[4].p, F[5].p};
  T* eo[3] = {G[0].p, G[1].p, G[2].p};
  T* ho[3] = {G[3].p, G[4].p, G[5].p};
  const T* cbs[3] = {C[0].p, C[1].p, C[2].p};
  const T* dbs[3] = {C[3].p, C[4].p, C[5].p};
  const int src[4] = {sp[0], sp[1], sp[2], src_comp};
  double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int l = 0; l < T_blk; ++l) vals[l] = src_val(t + l);
  if (CE4.p)
    K_OK(tb3d(ei, hi, eo, ho, cbs, dbs, cb, db, N[0], N[1], N[2], boxes, T_blk, src, vals, st, CE4.p, ebox));
  else
    K_OK(tb3d(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], N[1], N[2], boxes, T_blk, src,
              vals, st));
  for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
}

// n steps from step t0 through the planned passes (hybrid 3D / 2D, blocked,
// the resident 1D run) and single steps for what remains
template <typename T>
void NativeRun<T>::advance(int t0, int n) {
  int t = t0;
  // (with the Drude box in the passes a tail is a shorter pass too: the
  // stepped chain never holds the box's state)
  while (T_h > 1 && (n >= T_h || (dr_blk && n > 0))) {
    const int k = std::min(T_h, n);
    hybrid_pass(t, k);
    t += k;
    n -= k;
  }
  while (T2_h > 1 && n >= T2_h) {
    hybrid2d_pass(t);
    t += T2_h;
    n -= T2_h;
  }
  if (res1 && n > 0) {
    std::vector<T> hv(n);
    for (int l = 0; l < n; ++l) hv[l] = (T)src_val(t + l);
    Dev<T> dv;
    dv.alloc(n);
    HIP_OK(hipMemcpyAsync(dv.p, hv.data(), n * sizeof(T), hipMemcpyHostToDevice, st));
    const int b1[4] = {boxes[12], boxes[15], boxes[24], boxes[27]};
    K_OK(res1d(F[2].p, F[4].p, C[2].p, C[4].p, percell ? 1.0 : cb, percell ? 1.0 : db, N[0], b1, n, sp[0], dv.p, st));
    HIP_OK(hipStreamSynchronize(st));  // the table is freed on return
    return;
  }
  while (n > 0) {
    if (T2_blk > 1) {
      const int k = std::min(T2_blk, n);
      blocked2d_pass(t, k);
      t += k;
      n -= k;
    } else if (T_blk > 1 && n >= T_blk) {
      blocked3d_pass(t);
      t += T_blk;
      n -= T_blk;
    } else {
      step(t);
      ++t;
      --n;
    }
  }
}

// ==================================================================== run loop

// NTFF diagram after every step t with (t - 1) % ntffStep == 0, for the
// fields of step t - 1 (the Python driver's periodic hook, runner.py)
template <typename T>
void NativeRun<T>::ntff_report(int t) {
  HIP_OK(hipStreamSynchronize(st));
  fptrs();
  const int nbox[3] = {s.ntffSizeX, s.ntffSizeY, s.ntffSizeZ};
  const std::vector<double> phis = native_phys::reference_angles();
  const std::vector<double> p =
      native_phys::ntff_power<T>(Fp, N, nbox, dx, s.sourceWaveLength, s.incidentWaveAngle1 * (kPi / 180.0), phis);
  for (size_t q = 0; q < phis.size(); ++q)
    std::printf("=== t=%u, inc angle=%f; angle %f === %.17g \n", (unsigned)t, s.incidentWaveAngle2 * (kPi / 180.0),
                phis[q], p[q]);
}

template <typename T>
void NativeRun<T>::run_steps(int t0, int n) {
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

// --checkpoint-step P: a checkpoint after every step t with t % P == 0 (the
// Python driver's periodic hook), the passes ending there; the checkpoint I/O
// time (host wall clock, the device idle) is kept out of the reported
// stepping rate, as the Python driver's phase timers do
template <typename T>
void NativeRun<T>::run_ckpt(int t, int n) {
  const int P = s.checkpointDir.empty() ? 0 : s.checkpointStep;
  if (P <= 0) {
    run_steps(t, n);
    return;
  }
  const int end = t + n;
  while (t < end) {
    const int nxt = std::min(end, (t / P + 1) * P);
    run_steps(t, nxt - t);
    t = nxt;
    if (t % P == 0) {
      HIP_OK(hipStreamSynchronize(st));
      const auto c0 = std::chrono::steady_clock::now();
      if (!ckpt_save<T>(s, scheme, N, present, F, t, dx, dt)) {
        std::fprintf(stderr, "fdtd3d: cannot write the checkpoint to %s\n", s.checkpointDir.c_str());
        std::exit(1);
      }
      ckpt_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
    }
  }
}

// every array that carries state between steps, in logical order (the
// current F / D level lists, whatever the pointer swaps did): the amplitude
// mode's snapshot of a check period
template <typename T>
std::vector<std::pair<void*, size_t>> NativeRun<T>::amp_state() {
  std::vector<std::pair<void*, size_t>> v;
  for (int c = 0; c < 6; ++c)
    if (present[c]) v.push_back({F[c].p, cells * sizeof(T)});
  if (tfsf) {
    v.push_back({tft.einc.p, (size_t)tft.nline * sizeof(T)});
    v.push_back({tft.hinc.p, (size_t)tft.nline * sizeof(T)});
  }
  for (auto* d : cpt.keep) v.push_back({d->p, d->n * sizeof(T)});
  for (const Slab2d<T>& sl : p2.slabs)
    v.push_back({sl.psi, (size_t)(sl.pbox[3] - sl.pbox[0]) * (sl.pbox[4] - sl.pbox[1]) * (sl.pbox[5] - sl.pbox[2]) *
                             sizeof(T)});
  for (int c = 0; c < 6; ++c) {
    for (int l = 0; l < 2; ++l)
      if (p2.D[c][l]) v.push_back({p2.D[c][l], cells * sizeof(T)});
    for (const auto& lv : upt.D[c])
      for (size_t q = 0; q < lv.size(); ++q) v.push_back({lv[q], upt.rvol[q] * sizeof(T)});
    for (const auto& lv : upt.D1[c])
      for (size_t q = 0; q < lv.size(); ++q)
        if (lv[q]) v.push_back({lv[q], upt.rvol[q] * sizeof(T)});
  }
  return v;
}

template <typename T>
void NativeRun<T>::report(double sec, int t_end, int steps, int warm) const {
  std::printf("Total time = %f seconds\n", sec);
  if (ckpt_ms > 0) std::printf("Checkpoint I/O = %f seconds (not in the total)\n", ckpt_ms / 1e3);
  std::printf("Dimension: %d\n", dim);
  if (dim == 3)
    std::printf("Grid size: %dx%dx%d\n", N[0], N[1], N[2]);
  else if (dim == 2)
    std::printf("Grid size: %dx%d\n", N[0], N[1]);
  else
    std::printf("Grid size: %d\n", N[0]);
  const int timed = steps - warm + ampm.taken;
  std::printf("Number of time steps: %d (%d timed after %d warm-up)\n\n", t_end, timed, warm);
  std::printf("Value type: %s\n", Api<T>::name);
  if (s.doUseComplexFieldValues) std::printf("Complex field values: 1 (real and imaginary planes)\n");
  std::printf("\n-------- Details --------\n");
  std::printf("Parallel grid: 0\n");
  if (T2_h > 1)
    std::printf("Backend: native HIP, hybrid passes (2D blocked core, %d steps per pass; stepped %s%s shell)\n", T2_h,
                upml ? "UPML" : "CPML", tfsf ? " + TF/SF" : "");
  else if (T_h > 1)
    std::printf("Backend: native HIP, hybrid passes (blocked core, %d steps per pass; stepped %s%s shell%s)\n", T_h,
                upml ? "UPML" : (cpml ? "CPML" : "plain"), tfsf ? " + TF/SF" : "",
                dr_blk ? "; the Drude box inside the passes" : "");
  else if (T_blk > 1 || T2_blk > 1)
    std::printf("Backend: native HIP, temporally blocked kernel (%d steps per pass)\n", std::max(T_blk, T2_blk));
  else if (res1)
    std::printf("Backend: native HIP, register-resident 1D kernel (one launch per run)\n");
  else if (cpml || tfsf || upml)
    std::printf("Backend: native HIP, split kernels%s%s%s\n", cpml ? " with the CPML terms folded in" : "",
                upml ? " with the UPML / dispersive chain" : "", tfsf ? " + TF/SF corrections" : "");
  else
    std::printf("Backend: native HIP, %s kernels%s\n", use_fused ? "fused E+H" : "split", v4 ? " (float4)" : "");
  std::printf("Throughput: %.1f Mcells/s\n", cells * (double)timed / sec / 1e6);
  if (amp) {
    if (ampm.stable > 0)
      std::printf("Amplitude mode: stable after %d steps (%d amplitude steps taken)\n", ampm.stable, ampm.taken);
    else
      std::printf("Amplitude mode: stable state not reached after %d steps\n", ampm.taken);
  }
  if (s.doPrintJson)
    std::printf("{\"seconds\": %.6f, \"steps\": %d, \"mcells_per_s\": %.3f}\n", sec, timed,
                cells * (double)timed / sec / 1e6);
}

// --save-res (DAT / BMP of the final fields) and the final checkpoint
template <typename T>
bool NativeRun<T>::save_results(int t_end) {
  if (s.doSaveRes) {
    const char* names[6] = {"Ex", "Ey", "Ez", "Hx", "Hy", "Hz"};
    std::vector<T> host(cells);
    for (int c = 0; c < 6; ++c) {
      if (!present[c]) continue;
      HIP_OK(hipMemcpy(host.data(), F[c].p, cells * sizeof(T), hipMemcpyDeviceToHost));
      const std::string base = fdtd::grid_file_name(t_end, 0, names[c], s.outputDir == "." ? "" : s.outputDir);
      if (s.saveAsDAT) fdtd::write_dat(base + ".dat", host.data(), cells * sizeof(T));
      if (s.saveAsBMP || !s.saveAsDAT) {
        // middle slice along z (3D) or the plane (2D) / line (1D)
        const int w = N[0], h = N[1];
        const int kz = dim == 3 ? N[2] / 2 : 0;
        std::vector<double> v((size_t)w * h);
        for (int i = 0; i < w; ++i)
          for (int j = 0; j < h; ++j) v[(size_t)i * h + j] = host[((size_t)i * N[1] + j) * N[2] + kz];
        const std::string name = dim == 3 ? base + std::to_string(kz) + "-Re.bmp" : base + "-Re.bmp";
        fdtd::write_bmp(name, v, w, h, s.dumperPalette);
      }
    }
  }
  if (!s.checkpointDir.empty() && !ckpt_save<T>(s, scheme, N, present, F, t_end, dx, dt)) {
    std::fprintf(stderr, "fdtd3d: cannot write the checkpoint to %s\n", s.checkpointDir.c_str());
    return false;
  }
  return true;
}

template <typename T>
bool NativeRun<T>::prepare() {
  setup_fields();
  setup_absorbers();
  setup_chain_regions();
  plan_drude();
  if (!setup_sources_and_modes()) return false;
  plan_blocking();
  setup_streams();
  // --load-from-file: the run continues from the checkpoint's step up to --time-steps
  t0_ = 0;
  if (!s.loadFromFile.empty()) {
    const long got = ckpt_load<T>(s, scheme, N, present, F);
    if (got < 0) return false;
    t0_ = (int)got;
  }
  steps_ = std::max(0, s.numTimeSteps - t0_);
  warm_ = std::max(0, std::min(s.warmupSteps, steps_));
  return true;
}

template <typename T>
void NativeRun<T>::run_timed() {
  const int t0 = t0_, steps = steps_, warm = warm_;
  run_ckpt(t0, warm);  // untimed (they advance the simulation)
  HIP_OK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, st));
  ckpt_ms = 0.0;  // warm-up checkpoints are outside the timed region anyway
  run_ckpt(t0 + warm, steps - warm);
  // amplitude mode (native_amp.h): after the regular steps, check periods
  // until a step changes no running maximum
  int t_end = t0 + steps;
  if (amp) {
    // blocked amplitude passes: 3D vacuum fp32 float4 rows, no absorbing layer / TF/SF / NTFF
    const bool blocked = scheme == "3d" && sizeof(T) == 4 && v4 && !percell && !cpml && !upml && !tfsf && !ntff &&
                         ampm.line_n > 0 && !s.doUseSplitKernels;
    t_end = ampm.run(s, N, active, present, boxes, F, G, blocked, cb, db, st, t0 + steps,
                     [this](int t) { return src_val(t); }, [this](int t) { step(t); },
                     [this]() { return amp_state(); });
  }
  HIP_OK(hipEventRecord(e1, st));
  HIP_OK(hipEventSynchronize(e1));
  HIP_OK(hipGetLastError());
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  HIP_OK(hipEventDestroy(e0));
  HIP_OK(hipEventDestroy(e1));
  sec_ = std::max(0.0, (ms - ckpt_ms) / 1e3);
  t_end_ = t_end;
}

template <typename T>
int NativeRun<T>::main() {
  if (!prepare()) return 1;
  run_timed();
  report_run();
  return save_results(t_end_) ? 0 : 1;
}

// a complex run's outputs (this = the real plane): DAT files of interleaved
// (real, imaginary) values -- the reference's std::complex<T> layout, as
// io/dat.py writes them -- and -Re / -Im / -Mod images of the middle slice
template <typename T>
bool NativeRun<T>::save_complex(const NativeRun<T>& im) const {
  if (!s.doSaveRes) return true;
  const char* names[6] = {"Ex", "Ey", "Ez", "Hx", "Hy", "Hz"};
  std::vector<T> re(cells), ip(cells), both(2 * cells);
  for (int c = 0; c < 6; ++c) {
    if (!present[c]) continue;
    HIP_OK(hipMemcpy(re.data(), F[c].p, cells * sizeof(T), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(ip.data(), im.F[c].p, cells * sizeof(T), hipMemcpyDeviceToHost));
    for (size_t q = 0; q < cells; ++q) {
      both[2 * q] = re[q];
      both[2 * q + 1] = ip[q];
    }
    const std::string base = fdtd::grid_file_name(t_end_, 0, names[c], s.outputDir == "." ? "" : s.outputDir);
    if (s.saveAsDAT && !fdtd::write_dat(base + ".dat", both.data(), both.size() * sizeof(T))) return false;
    if (s.saveAsBMP || !s.saveAsDAT) {
      const int w = N[0], h = N[1];
      const int kz = dim == 3 ? N[2] / 2 : 0;
      std::vector<double> vr((size_t)w * h), vi((size_t)w * h), vm((size_t)w * h);
      for (int i = 0; i < w; ++i)
        for (int j = 0; j < h; ++j) {
          const size_t o = ((size_t)i * N[1] + j) * N[2] + kz, q = (size_t)i * h + j;
          vr[q] = re[o];
          vi[q] = ip[o];
          vm[q] = std::sqrt(vr[q] * vr[q] + vi[q] * vi[q]);
        }
      const std::string stem = dim == 3 ? base + std::to_string(kz) : base;
      fdtd::write_bmp(stem + "-Re.bmp", vr, w, h, s.dumperPalette);
      fdtd::write_bmp(stem + "-Im.bmp", vi, w, h, s.dumperPalette);
      fdtd::write_bmp(stem + "-Mod.bmp", vm, w, h, s.dumperPalette);
    }
  }
  return true;
}

}  // namespace
