// native_multi.h -- --parallel-grid x-slab decompositions driven from one process.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "capi.h"
#include "host_native.h"
#include "settings_native.h"
#include "native_api.h"
#include "native_setup.h"

// Part of the native driver: included by main.cpp only (one translation unit),
// hence the unnamed namespace.
namespace {

// ------------------------------------------------------------ multi-GPU
// --parallel-grid: the 3D grid split into x slabs over P ranks, all driven
// by this one process (rank r on device r % devices; --topology-sizex P, or
// one rank per visible GPU).  x is the slowest axis, so a rank's T ghost
// planes on each side are contiguous: no pack / unpack kernels, one
// device-to-device (xGMI peer) copy per field and side.  Every T steps each
// rank runs the temporally blocked kernel over its owned planes (reading the
// T-deep ghosts, the pass's dependency cone), then pulls its neighbours'
// fresh boundary planes on its own stream; events order the passes and the
// pulls across streams (a rank's next pass waits for its neighbours' pulls
// from the buffer it is about to overwrite).  Point-to-point and nearest-
// neighbour only, the shape of the node's xGMI links.  Plain Yee media
// (vacuum / dielectric sphere) with the point source; the reference's MPI
// grid: Source/Grid/ParallelGrid.cpp:1600-1823 (exchange), :2161-2194.
template <typename T>
struct XRank {
  int dev = 0;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr, copied = nullptr;
  int lo = 0, hi = 0, gl = 0, gh = 0, x0 = 0, nx = 0;
  Dev<T> F[6], G[6], C[6];
  int boxes[36];
};

template <typename T>
int run_multi(const fdtd::Settings& s) {
  fdtd::Int3 N = {s.sizeX, s.sizeY, s.sizeZ};
  const std::vector<int> active = {0, 1, 2};
  const double dx = s.gridStep, courant = s.courantNum;
  const double dt = dx * courant / kC;
  const double freq = kC / s.sourceWaveLength;
  const double cb = dt / (kEps0 * dx), db = dt / (kMu0 * dx);
  const bool percell = s.scene != "vacuum";
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  const int P = s.topologySizeX > 1 ? s.topologySizeX : ndev;
  const int T_max = sizeof(T) == 4 ? fdtd_tb_max_steps() : fdtd_tb64_max_steps();
  const int TB = std::max(1, std::min(T_max, s.timeBlock <= 0 ? (sizeof(T) == 4 ? 5 : 4) : s.timeBlock));
  if (sizeof(T) == 4 && N[2] % 4 != 0) {
    std::fprintf(stderr, "fdtd3d (native): fp32 parallel grids need sizez %% 4 == 0 (float4 rows)\n");
    return 2;
  }
  if (N[0] / P < TB) {
    std::fprintf(stderr, "fdtd3d (native): %d x planes over %d ranks leave fewer than %d planes per rank\n", N[0], P,
                 TB);
    return 2;
  }
  const size_t plane = (size_t)N[1] * N[2];
  std::vector<XRank<T>> R(P);
  for (int r = 0, x = 0; r < P; ++r) {
    XRank<T>& q = R[r];
    q.dev = r % ndev;
    q.lo = x;
    q.hi = x + N[0] / P + (r < N[0] % P ? 1 : 0);
    x = q.hi;
    q.gl = r > 0 ? TB : 0;
    q.gh = r < P - 1 ? TB : 0;
    q.x0 = q.lo - q.gl;
    q.nx = q.hi - q.lo + q.gl + q.gh;
    HIP_OK(hipSetDevice(q.dev));
    HIP_OK(hipStreamCreate(&q.st));
    HIP_OK(hipEventCreateWithFlags(&q.done, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&q.copied, hipEventDisableTiming));
    const size_t n = (size_t)q.nx * plane;
    for (int c = 0; c < 6; ++c) {
      q.F[c].alloc(n);
      q.G[c].alloc(n);
    }
    // update boxes in local indices: the global range of each component
    // clipped to the rank's planes (ghosts included)
    for (int c = 0; c < 6; ++c) {
      fdtd::Int3 glo, ghi;
      fdtd::global_range(c, N, active, glo, ghi);
      q.boxes[6 * c] = std::max(glo[0], q.x0) - q.x0;
      q.boxes[6 * c + 3] = std::min(ghi[0], q.x0 + q.nx) - q.x0;
      for (int a = 1; a < 3; ++a) {
        q.boxes[6 * c + a] = glo[a];
        q.boxes[6 * c + 3 + a] = ghi[a];
      }
    }
    if (percell) {
      // per-cell E coefficients of the dielectric sphere (2-point eps
      // averages, as the single-rank path), H on the scalar db
      const double ctr[3] = {s.sphereCenterX, s.sphereCenterY, s.sphereCenterZ};
      std::vector<T> host(n);
      for (int c = 0; c < 3; ++c) {
        const int di = c == 0, dj = c == 1, dk = c == 2;
        for (int li = 0; li < q.nx; ++li)
          for (int j = 0; j < N[1]; ++j)
            for (int k = 0; k < N[2]; ++k) {
              const int i = q.x0 + li;
              const double a = sphere_eps(i + 0.5, j + 0.5, k + 0.5, ctr, s.sphereRadius, s.sphereEps);
              const double b = sphere_eps(i + di + 0.5, j + dj + 0.5, k + dk + 0.5, ctr, s.sphereRadius, s.sphereEps);
              host[((size_t)li * N[1] + j) * N[2] + k] = (T)(cb * 2.0 / (a + b));
            }
        q.C[c].alloc(n);
        HIP_OK(hipMemcpy(q.C[c].p, host.data(), n * sizeof(T), hipMemcpyHostToDevice));
      }
    }
  }
  // peer access between neighbouring devices (xGMI)
  for (int r = 0; r + 1 < P; ++r)
    if (R[r].dev != R[r + 1].dev) {
      for (int d = 0; d < 2; ++d) {
        const int a = R[r + d].dev, b = R[r + 1 - d].dev;
        int ok = 0;
        HIP_OK(hipDeviceCanAccessPeer(&ok, a, b));
        if (ok) {
          HIP_OK(hipSetDevice(a));
          const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
          if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIP_OK(e);
        }
      }
    }
  (void)hipGetLastError();
  const fdtd::Int3 sp = {N[0] / 2, N[1] / 2, N[2] / 2};
  auto src_val = [&](int t) {
    if (s.sourceType == "gaussian") return std::exp(-std::pow((t - s.gaussianDelay) / s.gaussianWidth, 2));
    return std::sin(dt * t * 2 * kPi * freq);
  };
  bool first = true;
  // k steps on every rank, then the ghost pulls
  auto pass = [&](int t, int k) {
    for (int r = 0; r < P; ++r) {
      XRank<T>& q = R[r];
      HIP_OK(hipSetDevice(q.dev));
      if (!first) {
        // the neighbours' pulls from this rank's (old) F are done before the
        // pass overwrites it as its output buffer
        if (r > 0) HIP_OK(hipStreamWaitEvent(q.st, R[r - 1].copied, 0));
        if (r < P - 1) HIP_OK(hipStreamWaitEvent(q.st, R[r + 1].copied, 0));
      }
      const T* ei[3] = {q.F[0].p, q.F[1].p, q.F[2].p};
      const T* hi[3] = {q.F[3].p, q.F[4].p, q.F[5].p};
      T* eo[3] = {q.G[0].p, q.G[1].p, q.G[2].p};
      T* ho[3] = {q.G[3].p, q.G[4].p, q.G[5].p};
      const T* cbs[3] = {q.C[0].p, q.C[1].p, q.C[2].p};
      const T* dbs[3] = {nullptr, nullptr, nullptr};
      // every rank whose planes (ghosts included) hold the source plane sets
      // the hard source: a neighbour's redundant ghost-plane levels need it
      const bool has = sp[0] >= q.x0 && sp[0] < q.x0 + q.nx;
      const int src[4] = {sp[0] - q.x0, sp[1], sp[2], has ? 2 : -1};
      double vals[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int l = 0; l < k; ++l) vals[l] = src_val(t + l);
      const int ob[6] = {q.lo - q.x0, 0, 0, q.hi - q.x0, N[1], N[2]};
      if constexpr (sizeof(T) == 4)
        K_OK(fdtd_tb3d_v4_f32(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, db, q.nx, N[1], N[2], q.boxes, ob, 0, k,
                              src, vals, q.st));
      else
        K_OK(fdtd_tb3d_f64(ei, hi, eo, ho, cbs, dbs, percell ? 1.0 : cb, db, q.nx, N[1], N[2], q.boxes, ob, 0, k, src,
                           vals, q.st));
      for (int c = 0; c < 6; ++c) std::swap(q.F[c].p, q.G[c].p);
      HIP_OK(hipEventRecord(q.done, q.st));
    }
    for (int r = 0; r < P; ++r) {
      XRank<T>& q = R[r];
      HIP_OK(hipSetDevice(q.dev));
      for (int side = 0; side < 2; ++side) {
        const int nb = side == 0 ? r - 1 : r + 1;
        if (nb < 0 || nb >= P) continue;
        const XRank<T>& o = R[nb];
        HIP_OK(hipStreamWaitEvent(q.st, o.done, 0));
        // low ghosts <- the lower neighbour's top T owned planes; high ghosts
        // <- the upper neighbour's bottom T owned planes
        const int src_x = side == 0 ? o.hi - TB : o.lo;
        const int dst_x = side == 0 ? q.lo - TB : q.hi;
        const size_t bytes = (size_t)TB * plane * sizeof(T);
        for (int c = 0; c < 6; ++c) {
          T* dst = q.F[c].p + (size_t)(dst_x - q.x0) * plane;
          const T* srcp = o.F[c].p + (size_t)(src_x - o.x0) * plane;
          if (o.dev == q.dev)
            HIP_OK(hipMemcpyAsync(dst, srcp, bytes, hipMemcpyDeviceToDevice, q.st));
          else
            HIP_OK(hipMemcpyPeerAsync(dst, q.dev, srcp, o.dev, bytes, q.st));
        }
      }
      HIP_OK(hipEventRecord(q.copied, q.st));
    }
    first = false;
  };
  auto advance = [&](int t0, int n) {
    int t = t0;
    while (n > 0) {
      const int k = std::min(TB, n);
      pass(t, k);
      t += k;
      n -= k;
    }
  };
  auto sync_all = [&]() {
    for (int r = 0; r < P; ++r) {
      HIP_OK(hipSetDevice(R[r].dev));
      HIP_OK(hipStreamSynchronize(R[r].st));
    }
  };
  const int steps = s.numTimeSteps;
  const int warm = std::max(0, std::min(s.warmupSteps, steps));
  advance(0, warm);
  sync_all();
  const auto c0 = std::chrono::steady_clock::now();
  advance(warm, steps - warm);
  sync_all();
  HIP_OK(hipGetLastError());
  const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
  const double cells = (double)N[0] * N[1] * N[2];
  const int timed = steps - warm;
  std::printf("Total time = %f seconds\n", sec);
  std::printf("Dimension: 3\n");
  std::printf("Grid size: %dx%dx%d\n", N[0], N[1], N[2]);
  std::printf("Number of time steps: %d (%d timed after %d warm-up)\n\n", steps, timed, warm);
  std::printf("Value type: %s\n", Api<T>::name);
  std::printf("\n-------- Details --------\n");
  std::printf("Parallel grid: 1\n");
  std::printf("Number of processes: %d (ranks of one process on %d device%s)\n", P, std::min(P, ndev),
              std::min(P, ndev) > 1 ? "s" : "");
  std::printf("Parallel grid scheme: X (topology %dx1x1)\n", P);
  std::printf("Buffer size: %d\n", TB);
  std::printf("Backend: native HIP, temporally blocked kernel (%d steps per pass), x-slab ghost planes by peer copies\n",
              TB);
  std::printf("Throughput: %.1f Mcells/s\n", cells * timed / sec / 1e6);
  if (s.doPrintJson)
    std::printf("{\"seconds\": %.6f, \"steps\": %d, \"mcells_per_s\": %.3f, \"ranks\": %d}\n", sec, timed,
                cells * timed / sec / 1e6, P);
  if (s.doSaveRes) {
    const char* names[6] = {"Ex", "Ey", "Ez", "Hx", "Hy", "Hz"};
    std::vector<T> host((size_t)N[0] * plane);
    for (int c = 0; c < 6; ++c) {
      for (int r = 0; r < P; ++r) {
        const XRank<T>& q = R[r];
        HIP_OK(hipSetDevice(q.dev));
        HIP_OK(hipMemcpy(host.data() + (size_t)q.lo * plane, q.F[c].p + (size_t)q.gl * plane,
                         (size_t)(q.hi - q.lo) * plane * sizeof(T), hipMemcpyDeviceToHost));
      }
      const std::string base = fdtd::grid_file_name(steps, 0, names[c], s.outputDir == "." ? "" : s.outputDir);
      if (s.saveAsDAT) fdtd::write_dat(base + ".dat", host.data(), host.size() * sizeof(T));
      if (s.saveAsBMP || !s.saveAsDAT) {
        const int kz = N[2] / 2;
        std::vector<double> v((size_t)N[0] * N[1]);
        for (int i = 0; i < N[0]; ++i)
          for (int j = 0; j < N[1]; ++j) v[(size_t)i * N[1] + j] = host[((size_t)i * N[1] + j) * N[2] + kz];
        fdtd::write_bmp(base + std::to_string(kz) + "-Re.bmp", v, N[0], N[1], s.dumperPalette);
      }
    }
  }
  for (auto& q : R) {
    HIP_OK(hipSetDevice(q.dev));
    for (int c = 0; c < 6; ++c) {  // freed with the rank's device current
      q.F[c].reset();
      q.G[c].reset();
      q.C[c].reset();
    }
    HIP_OK(hipEventDestroy(q.done));
    HIP_OK(hipEventDestroy(q.copied));
    HIP_OK(hipStreamDestroy(q.st));
  }
  return 0;
}

}  // namespace
