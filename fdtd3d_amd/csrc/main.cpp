// fdtd3d -- standalone native driver (no Python): command line -> device
// fields -> HIP kernels -> timing report, the counterpart of the reference's
// Source/main.cpp built directly on libfdtd3d_hip's C ABI.
//
// Covers the plain Yee solvers (1D, 2D TMz/TEz, 3D) on one GPU with the
// vacuum / dielectric-sphere scenes and the hard point source, fp32 or fp64,
// fused or split 3D kernels, CPML absorbing layers in 3D fp32 or fp64 (--use-pml
// --pml-type cpml; with hybrid passes -- blocked core, stepped shell -- like
// the Python driver's automatic plan; z sizes not divisible by 4 on the scalar
// kernels + generic slab corrections), the UPML in the reference's D/B form and Drude / Lorentz
// spheres (--use-metamaterials, scene drude-sphere) in 3D through the fused
// chain kernel, TF/SF plane waves in 3D, the NTFF scattered power diagram
// (--use-ntff) and DAT/BMP output of the final fields (native_physics.h).
// 2D CPML / UPML and TF/SF (generic slab and chain kernels), amplitude mode
// (running maxima folded into blocked passes for 3D vacuum fp32, a fused
// amplitude kernel after each step otherwise), checkpoints / resume of
// plain-media runs in the Python driver's format (--checkpoint-dir,
// --load-from-file) and --parallel-grid decompositions (any x / y / z rank
// grid; 2D x / y, 1D x) over the node's GPUs from one process (run_multi): 3D plain media on
// blocked passes; CPML, the UPML, Drude / Lorentz spheres, TF/SF and
// amplitude mode on the split half steps; the NTFF diagram and plain-media
// checkpoints from the gathered grid.  Complex fields (one GPU) as two real
// planes.  What this binary does not run (complex fields with amplitude mode,
// NTFF, checkpoints or parallel grids) goes through the Python driver (python
// -m fdtd3d_amd), which shares the kernels; asking this binary for it is an
// error, never a silent fallback.
#include <hip/hip_runtime.h>

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <array>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

#include "capi.h"
#include "host_native.h"
#include "native_physics.h"
#include "settings_native.h"

#include "native_api.h"
#include "native_setup.h"
#include "native_ckpt.h"
#include "native_amp.h"
#include "native_lowdim.h"
#include "native_run.h"

namespace {


// one GPU: the stages of native_run.h (set-up, pass plans, the run loop, the report)
template <typename T>
int run(const fdtd::Settings& s) {
  if (s.doUseComplexFieldValues) {
    // complex fields (the reference's COMPLEX_FIELD_VALUES): the real and the
    // imaginary plane step as two real runs with the sin / cos source
    // (models/scheme.py planes); the rate counts both planes' time
    NativeRun<T> re(s, 0), im(s, 1);
    if (!re.prepare() || !im.prepare()) return 1;
    re.run_timed();
    im.run_timed();
    re.report_run(im.seconds());
    return re.save_complex(im) ? 0 : 1;
  }
  NativeRun<T> r(s);
  return r.main();
}

}  // namespace

#include "native_multi.h"


int main(int argc, char** argv) {
  fdtd::Settings s;
  int st = s.parse(argc, argv, true, 1);
  if (st == fdtd::SETTINGS_BREAK) {
    std::fputs(s.message.c_str(), stdout);
    return 0;
  }
  if (st != fdtd::SETTINGS_OK) {
    std::fputs(s.message.c_str(), stdout);
    return st;
  }
  if (s.validate() != fdtd::SETTINGS_OK) {
    std::fprintf(stdout, "ERROR: %s\n", s.message.c_str());
    return 1;
  }
  if (!native_supported(s)) {
    std::fprintf(stderr,
                 "fdtd3d (native): decomposed 3D CPML outside whole 4-cell z rows, PML / TF/SF in 1D, TF/SF boxes reaching "
                 "the UPML, metamaterials outside the 3D drude-sphere scene, amplitude mode with NTFF, parallel "
                 "grids with NTFF in 2D, checkpoints beyond plain media, and complex fields with amplitude mode, "
                 "NTFF, checkpoints or parallel grids run through the Python driver: python -m fdtd3d_amd <same options>\n");
    return 2;
  }
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  if (ndev < 1) {
    std::fprintf(stderr, "no HIP device\n");
    return 1;
  }
  if (s.doUseParallelGrid) return s.valueType == "f32" ? run_multi<float>(s) : run_multi<double>(s);
  HIP_OK(hipSetDevice(0 % (s.numCudaGPUs > 0 ? s.numCudaGPUs : 1)));
  return s.valueType == "f32" ? run<float>(s) : run<double>(s);
}
