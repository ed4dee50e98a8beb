// native_amp.h -- the native driver's amplitude (steady-state) mode: running
// maxima of every component, per-step changed counts and the stop rule of
// models/scheme.py perform_amplitude_steps (reference Scheme3D.cpp:2945-3333).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <utility>
#include <vector>

#include "capi.h"
#include "host_native.h"
#include "settings_native.h"
#include "native_api.h"
#include "native_setup.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
namespace {

template <typename T>
struct AmpMode {
  Dev<T> AMP;           // running maxima, one [x][6][y][z] buffer (the blocked amplitude kernel's layout)
  Dev<unsigned> CNT;    // changed counts of the steps of one check period
  Dev<long long> LINE;  // cells of the Ez z-line source
  int line_n = 0, line_k0 = 0;
  bool active = false;  // inside the amplitude phase: the z line replaces the point source
  int taken = 0, stable = -1;

  // the Ez z-line source at (Nx/8, Ny/2, k outside the z PML) of 3D runs with
  // a point source (Scheme3D.cpp:2995-3013)
  void init(const fdtd::Settings& s, const fdtd::Int3& N, bool line_src) {
    const size_t plane = (size_t)N[1] * N[2];
    AMP.alloc((size_t)N[0] * 6 * plane);
    CNT.alloc(std::max(1, s.amplitudeCheckSteps));
    if (!line_src) return;
    line_k0 = s.doUsePML ? s.pmlSizeZ : 0;
    std::vector<long long> offs;
    for (int k = line_k0; k < N[2] - line_k0; ++k) offs.push_back(((long long)(N[0] / 8) * N[1] + N[1] / 2) * N[2] + k);
    line_n = (int)offs.size();
    if (line_n > 0) {
      LINE.alloc(offs.size());
      HIP_OK(hipMemcpy(LINE.p, offs.data(), offs.size() * sizeof(long long), hipMemcpyHostToDevice));
    }
  }

  // The amplitude phase from step t: check periods of K steps whose changed-
  // cell counts accumulate on the device, read once per period; the run ends
  // with the period in which a step (after the first) changed no running
  // maximum, or after --amplitude-time-steps steps.  `blocked`: 3D vacuum fp32
  // float4 rows with the z line, the maxima folded into blocked passes
  // (tb3d_mr.h AmpDev); otherwise `step` + the fused amplitude kernel.
  // `state` lists every other array that carries state between steps (the
  // near-convergence snapshot).  Returns the last step.
  int run(const fdtd::Settings& s, const fdtd::Int3& N, const std::vector<int>& axes, const bool* present,
          const int* boxes, Dev<T>* F, Dev<T>* G, bool blocked, double cb, double db, hipStream_t st, int t,
          const std::function<double(int)>& src_val, const std::function<void(int)>& step,
          const std::function<std::vector<std::pair<void*, size_t>>()>& state) {
    active = true;
    const size_t cells = (size_t)N[0] * N[1] * N[2], plane = (size_t)N[1] * N[2];
    const int K = std::max(1, s.amplitudeCheckSteps);
    // amplitude box per component: its update box minus the PML cells
    // (Scheme3D.cpp:3016-3030); only present components
    int ab[36] = {}, na = 0;
    const T* af[6];
    T* aa[6];
    for (int c = 0; c < 6; ++c) {
      int* b = ab + 6 * c;
      for (int q = 0; q < 6; ++q) b[q] = boxes[6 * c + q];
      const int left[3] = {s.doUsePML ? s.pmlSizeX : 0, s.doUsePML ? s.pmlSizeY : 0, s.doUsePML ? s.pmlSizeZ : 0};
      for (int a : axes) {
        const int right = N[a] - left[a];
        if (left[a] == right) continue;
        b[a] = std::max(b[a], (int)std::ceil(left[a] - kMinFP[c][a]));
        b[3 + a] = std::min(b[3 + a], (int)std::ceil(right - kMinFP[c][a]));
      }
    }
    int abp[36];
    for (int c = 0; c < 6; ++c)
      if (present[c]) {
        af[na] = F[c].p;
        aa[na] = AMP.p + c * plane;
        std::memcpy(abp + 6 * na, ab + 6 * c, 6 * sizeof(int));
        ++na;
      }
    const int Ta = blocked ? 3 : 1;
    if (Ta > 1)
      for (int c = 0; c < 6; ++c)
        if (!G[c].p) G[c].alloc(cells);
    std::vector<unsigned> got(K);
    // one check period of n steps: blocked amplitude passes where they apply,
    // per-step stepping + the fused amplitude kernel otherwise; leaves the
    // per-step changed counts in `got`
    auto period = [&](int n) {
      HIP_OK(hipMemsetAsync(CNT.p, 0, K * sizeof(unsigned), st));
      int q = 0;
      while (q < n) {
        if (Ta > 1 && n - q >= 2) {
          if constexpr (sizeof(T) == 4) {
            const int k = std::min(Ta, n - q);
            const T* ei[3] = {F[0].p, F[1].p, F[2].p};
            const T* hi[3] = {F[3].p, F[4].p, F[5].p};
            T* eo[3] = {G[0].p, G[1].p, G[2].p};
            T* ho[3] = {G[3].p, G[4].p, G[5].p};
            const int ob[6] = {0, 0, 0, N[0], N[1], N[2]};
            const int src5[5] = {N[0] / 8, N[1] / 2, line_k0, 2, line_k0 + line_n};
            double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int l = 0; l < k; ++l) vals[l] = src_val(t + l);
            K_OK(fdtd_tb3d_amp_f32(ei, hi, eo, ho, cb, db, N[0], N[1], N[2], boxes, ob, 0, k, src5, vals, aa, ab,
                                   0.001, CNT.p + q, st));
            for (int c = 0; c < 6; ++c) std::swap(F[c].p, G[c].p);
            for (int c = 0; c < 6; ++c) af[c] = F[c].p;
            q += k;
            t += k;
            continue;
          }
        }
        step(t);
        K_OK(amp_many(af, aa, na, N[1], N[2], abp, (long long)(6 * plane), 0.001, CNT.p + q, st));
        ++q;
        ++t;
      }
      HIP_OK(hipMemcpyAsync(got.data(), CNT.p, n * sizeof(unsigned), hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
    };
    // every array that carries state between steps, in logical order (the
    // current F / D level lists, whatever the pointer swaps did)
    auto all_state = [&]() {
      auto v = state();
      v.push_back({AMP.p, (size_t)N[0] * 6 * plane * sizeof(T)});
      return v;
    };
    long long acells = 0;
    for (int c = 0; c < na; ++c) {
      const int* b = abp + 6 * c;
      acells += (long long)std::max(0, b[3] - b[0]) * std::max(0, b[4] - b[1]) * std::max(0, b[5] - b[2]);
    }
    const long long near = std::max(1LL, (long long)(0.02 * (double)acells));
    Dev<char> SNAP;
    long long last = -1;
    bool done = false;
    while (!done && taken < s.numAmplitudeTimeSteps) {
      int n = std::min(K, s.numAmplitudeTimeSteps - taken);
      int t_snap = -1;
      if (n > 1 && last >= 0 && last <= near) {
        // near convergence: snapshot the state so the period can be redone
        // up to its stable step exactly
        const auto v = all_state();
        size_t total = 0;
        for (const auto& e : v) total += e.second;
        if (!SNAP.p) SNAP.alloc(total);
        size_t o = 0;
        for (const auto& e : v) {
          HIP_OK(hipMemcpyAsync(SNAP.p + o, e.first, e.second, hipMemcpyDeviceToDevice, st));
          o += e.second;
        }
        t_snap = t;
      }
      period(n);
      int first = -1;
      for (int r = 0; r < n && first < 0; ++r)
        if (got[r] == 0 && taken + r + 1 > 1) first = r;
      if (first < 0) {
        last = got[n - 1];
        taken += n;
        continue;
      }
      stable = taken + first + 1;
      if (first + 1 < n && t_snap >= 0) {
        // back to the period's start, then exactly the steps up to the stable one
        const auto v = all_state();
        size_t o = 0;
        for (const auto& e : v) {
          HIP_OK(hipMemcpyAsync(e.first, SNAP.p + o, e.second, hipMemcpyDeviceToDevice, st));
          o += e.second;
        }
        t = t_snap;
        n = first + 1;
        period(n);
      }
      taken += n;
      done = true;
    }
    active = false;
    return t;
  }
};

}  // namespace
