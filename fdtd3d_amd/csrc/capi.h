// C ABI of libfdtd3d_hip (the HIP kernels): prototypes for native callers.
// The Python side binds the same symbols through ctypes (ops/hip_ops.py).
#pragma once

#include <stdint.h>

extern "C" {
int fdtd_abi_version();

int fdtd_update_e3d_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy, const float* hz,
                        const float* cbx, const float* cby, const float* cbz, double cb, int nx, int ny, int nz,
                        const int* boxes, int xchunk, void* stream);
int fdtd_update_h3d_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey, const float* ez,
                        const float* dbx, const float* dby, const float* dbz, double db, int nx, int ny, int nz,
                        const int* boxes, int xchunk, void* stream);
int fdtd_update_e3d_f64(double* ex, double* ey, double* ez, const double* hx, const double* hy, const double* hz,
                        const double* cbx, const double* cby, const double* cbz, double cb, int nx, int ny, int nz,
                        const int* boxes, int xchunk, void* stream);
int fdtd_update_h3d_f64(double* hx, double* hy, double* hz, const double* ex, const double* ey, const double* ez,
                        const double* dbx, const double* dby, const double* dbz, double db, int nx, int ny, int nz,
                        const int* boxes, int xchunk, void* stream);
int fdtd_update_e3d_v4_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy, const float* hz,
                           const float* cbx, const float* cby, const float* cbz, double cb, int nx, int ny, int nz,
                           const int* boxes, int xchunk, void* stream);
// float4 split E / H updates with the CPML convolution terms folded in
// (yee3d_cpml.hip): cp = 9 x {psi_lo, psi_hi, b, c, 1/kappa - 1} per
// (component, axis), ci = 9 x {lo0, hi0, lo1, hi1}
int fdtd_update_e3d_cpml_v4_f32(float* ex, float* ey, float* ez, const float* hx, const float* hy, const float* hz,
                                const float* cbx, const float* cby, const float* cbz, double cb, int nx, int ny,
                                int nz, const int* boxes, int xchunk, const void* const* cp, const int* ci,
                                void* stream);
int fdtd_update_h3d_cpml_v4_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey, const float* ez,
                                const float* dbx, const float* dby, const float* dbz, double db, int nx, int ny,
                                int nz, const int* boxes, int xchunk, const void* const* cp, const int* ci,
                                void* stream);
// the same on 4-cell double groups
int fdtd_update_e3d_cpml_v4_f64(double* ex, double* ey, double* ez, const double* hx, const double* hy,
                                const double* hz, const double* cbx, const double* cby, const double* cbz, double cb,
                                int nx, int ny, int nz, const int* boxes, int xchunk, const void* const* cp,
                                const int* ci, void* stream);
int fdtd_update_h3d_cpml_v4_f64(double* hx, double* hy, double* hz, const double* ex, const double* ey,
                                const double* ez, const double* dbx, const double* dby, const double* dbz, double db,
                                int nx, int ny, int nz, const int* boxes, int xchunk, const void* const* cp,
                                const int* ci, void* stream);
// fused UPML / Drude chain of the three components of a kind (chain_kernels.hip):
// P = 24 pointers, S = 2 scalars, I = 25 ints per component (layout there)
int fdtd_chain_ints_per_comp();
int fdtd_chain_ptrs_per_comp();
int fdtd_chain3d_f32(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny, int nz,
                     void* stream);
int fdtd_chain3d_f64(const void* const* P, const double* S, const int* I, int drude, int kind_e, int ny, int nz,
                     void* stream);
// TF/SF: 1D incident line steps and the table-driven corrections
// (generic_kernels.hip; ijk may be null when the box holds every target)
int fdtd_inc_e_f32(float* einc, const float* hinc, int n, double c, double src, void* stream);
int fdtd_inc_e_f64(double* einc, const double* hinc, int n, double c, double src, void* stream);
int fdtd_inc_h_f32(const float* einc, float* hinc, int n, double c, void* stream);
int fdtd_inc_h_f64(const double* einc, double* hinc, int n, double c, void* stream);
int fdtd_tfsf_apply_f32(float* target, const long long* off, const long long* i0, const float* w0, const float* w1,
                        const float* coef, const int* ijk, int n, const float* inc, const int* box, void* stream);
int fdtd_tfsf_apply_f64(double* target, const long long* off, const long long* i0, const double* w0,
                        const double* w1, const double* coef, const int* ijk, int n, const double* inc,
                        const int* box, void* stream);
int fdtd_update_h3d_v4_f32(float* hx, float* hy, float* hz, const float* ex, const float* ey, const float* ez,
                           const float* dbx, const float* dby, const float* dbz, double db, int nx, int ny, int nz,
                           const int* boxes, int xchunk, void* stream);
int fdtd_fused3d_f32(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                     const float* const* cbs, const float* const* dbs, double cb, double db, int nx, int ny, int nz,
                     const int* boxes, int xchunk, long long src_off, int src_comp, double src_val, void* s);
int fdtd_fused3d_f64(const double* const* ein, const double* const* hin, double* const* eout,
                     double* const* hout, const double* const* cbs, const double* const* dbs, double cb, double db,
                     int nx, int ny, int nz, const int* boxes, int xchunk, long long src_off, int src_comp,
                     double src_val, void* s);
int fdtd_fused3d_v4_f32(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                        const float* const* cbs, const float* const* dbs, double cb, double db, int nx, int ny,
                        int nz, const int* boxes, int xchunk, long long src_off, int src_comp, double src_val,
                        void* s);

int fdtd_tb3d_v4_f32(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                     const float* const* cbs, const float* const* dbs, double cb, double db, int nx, int ny, int nz,
                     const int* boxes, const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                     void* stream);
int fdtd_tb_max_steps();
int fdtd_tb3d_ext_f32(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                      const void* ce4, const int* ebox, const void* ch4, const int* hbox, double cb, double db,
                      int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk, int steps,
                      const int* src, const double* src_vals, const void* tf, const float* gtab, void* stream);
int fdtd_box_pack_f32(float* const* fields, float* buf, int ncomp, int ny, int nz, const int* box, void* s);
int fdtd_box_pack_f64(double* const* fields, double* buf, int ncomp, int ny, int nz, const int* box, void* s);
int fdtd_box_unpack_f32(float* const* fields, const float* buf, int ncomp, int ny, int nz, const int* box, void* s);
int fdtd_box_unpack_f64(double* const* fields, const double* buf, int ncomp, int ny, int nz, const int* box, void* s);
int fdtd_box_xfer_f32(float* const* src, float* const* dst, int ncomp, int ny, int nz, const int* box, void* s);
int fdtd_box_xfer_f64(double* const* src, double* const* dst, int ncomp, int ny, int nz, const int* box, void* s);
int fdtd_tb3d_amp_f32(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                      double cb, double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                      int steps, const int* src, const double* src_vals, float* const* amp, const int* aboxes,
                      double accuracy, unsigned* counts, void* stream);
int fdtd_tb3d_drude_f32(const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                        double cb, double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                        int steps, const int* src, const double* src_vals, const int* bbox, void* const* sin,
                        void* const* sout, const void* lut, int nid, double cbd, void* stream);
int fdtd_tfdev_size();
int fdtd_tfsf_pass_f32(float* einc, float* hinc, int n, double ce, double ch, const double* src_vals, int steps,
                       int reach, int nE, int nH, const int* I0, const float* W0, const float* W1, const float* C,
                       float* gtab, void* stream);
int fdtd_tfsf_table_f32(const float* esrc, const float* hsrc, float* einc, float* hinc, int n, double ce, double ch,
                        const double* src_vals, int steps, int reach, int nE, int nH, const int* I0, const float* W0,
                        const float* W1, const float* C, float* gtab, void* stream);
int fdtd_tb3d_f64(const double* const* ein, const double* const* hin, double* const* eout, double* const* hout,
                  const double* const* cbs, const double* const* dbs, double cb, double db, int nx, int ny, int nz,
                  const int* boxes, const int* obox, int xchunk, int steps, const int* src, const double* src_vals,
                  void* stream);
int fdtd_tb3d_drude_f64(const double* const* ein, const double* const* hin, double* const* eout, double* const* hout,
                        double cb, double db, int nx, int ny, int nz, const int* boxes, const int* obox, int xchunk,
                        int steps, const int* src, const double* src_vals, const int* bbox, void* const* sin,
                        void* const* sout, const double* lut, int nid, double cbd, void* stream);
int fdtd_tfsf_pass_f64(double* einc, double* hinc, int n, double ce, double ch, const double* src_vals, int steps,
                       int reach, int nE, int nH, const int* I0, const double* W0, const double* W1, const double* C,
                       double* gtab, void* stream);
int fdtd_tfsf_table_f64(const double* esrc, const double* hsrc, double* einc, double* hinc, int n, double ce,
                        double ch, const double* src_vals, int steps, int reach, int nE, int nH, const int* I0,
                        const double* W0, const double* W1, const double* C, double* gtab, void* stream);
int fdtd_tb3d_tf_f64(const double* const* ein, const double* const* hin, double* const* eout, double* const* hout,
                     const double* const* cbs, const double* const* dbs, double cb, double db, int nx, int ny, int nz,
                     const int* boxes, const int* obox, int xchunk, int steps, const int* src,
                     const double* src_vals, const void* tf, const double* gtab, void* stream);
int fdtd_tb64_max_steps();
void fdtd_set_tb64_shape(int half);
int fdtd_tb2d_f32(int mode, const float* const* ein, const float* const* hin, float* const* eout, float* const* hout,
                  const float* const* cs, double cb, double db, int nx, int ny, const int* boxes, const int* obox,
                  int xchunk, int steps, const int* src, const double* src_vals, void* stream);
int fdtd_tb2d_max_steps();
int fdtd_tb2d_f64(int mode, const double* const* ein, const double* const* hin, double* const* eout,
                  double* const* hout, const double* const* cs, double cb, double db, int nx, int ny, const int* boxes,
                  const int* obox, int xchunk, int steps, const int* src, const double* src_vals, void* stream);
int fdtd_tb2d64_max_steps();
int fdtd_res1d_f32(float* ez, float* hy, const float* cbz, const float* dby, double cb, double db, int n,
                   const int* boxes, int nsteps, int src_i, const float* vals, void* s);
int fdtd_res1d_f64(double* ez, double* hy, const double* cbz, const double* dby, double cb, double db, int n,
                   const int* boxes, int nsteps, int src_i, const double* vals, void* s);
int fdtd_res1d_max_cells(int elem_bytes);

int fdtd_tmz_e_f32(float* ez, const float* hx, const float* hy, const float* cbz, double cb, int nx, int ny,
                   const int* box, int xchunk, void* s);
int fdtd_tmz_h_f32(float* hx, float* hy, const float* ez, const float* dbx, const float* dby, double db, int nx,
                   int ny, const int* boxes, int xchunk, void* s);
int fdtd_tez_e_f32(float* ex, float* ey, const float* hz, const float* cbx, const float* cby, double cb, int nx,
                   int ny, const int* boxes, int xchunk, void* s);
int fdtd_tez_h_f32(float* hz, const float* ex, const float* ey, const float* dbz, double db, int nx, int ny,
                   const int* box, int xchunk, void* s);
int fdtd_1d_e_f32(float* ez, const float* hy, const float* cbz, double cb, int lo, int hi, void* s);
int fdtd_1d_h_f32(float* hy, const float* ez, const float* dby, double db, int lo, int hi, void* s);
int fdtd_tmz_e_f64(double* ez, const double* hx, const double* hy, const double* cbz, double cb, int nx, int ny,
                   const int* box, int xchunk, void* s);
int fdtd_tmz_h_f64(double* hx, double* hy, const double* ez, const double* dbx, const double* dby, double db, int nx,
                   int ny, const int* boxes, int xchunk, void* s);
int fdtd_tez_e_f64(double* ex, double* ey, const double* hz, const double* cbx, const double* cby, double cb, int nx,
                   int ny, const int* boxes, int xchunk, void* s);
int fdtd_tez_h_f64(double* hz, const double* ex, const double* ey, const double* dbz, double db, int nx, int ny,
                   const int* box, int xchunk, void* s);
int fdtd_1d_e_f64(double* ez, const double* hy, const double* cbz, double cb, int lo, int hi, void* s);
int fdtd_1d_h_f64(double* hy, const double* ez, const double* dby, double db, int lo, int hi, void* s);

int fdtd_set_value_f32(float* f, long long off, double v, void* s);
int fdtd_set_value_f64(double* f, long long off, double v, void* s);
int fdtd_set_values_f32(float* f, const long long* offs, int n, double v, void* s);
int fdtd_set_values_f64(double* f, const long long* offs, int n, double v, void* s);

// generic building blocks (generic_kernels.hip): factored coefficients =
// scalar x (px, py, pz, cell) pointers; the 2D UPML chain and the CPML slabs
int fdtd_curl_general_f32(float* out, const float* inp, const float* const* srcs, const int* axes, const int* signs,
                          int nterms, int kind_e, double ca_s, const void* const* ca_p, double cb_s,
                          const void* const* cb_p, int ny, int nz, const int* box, void* s);
int fdtd_curl_general_f64(double* out, const double* inp, const double* const* srcs, const int* axes,
                          const int* signs, int nterms, int kind_e, double ca_s, const void* const* ca_p, double cb_s,
                          const void* const* cb_p, int ny, int nz, const int* box, void* s);
int fdtd_lincomb_f32(float* out, int nterms, const double* scalars, const void* const* ptrs, const float* const* xs,
                     int ny, int nz, const int* box, void* s);
int fdtd_lincomb_f64(double* out, int nterms, const double* scalars, const void* const* ptrs, const double* const* xs,
                     int ny, int nz, const int* box, void* s);
int fdtd_cpml_apply_f32(float* target, const float* src, float* psi, int axis, int sign, int kind_e, const float* bc,
                        const float* cc, const float* kc, double cb_s, const void* const* cb_p, int ny, int nz,
                        const int* box, const int* psi_box, void* s);
int fdtd_cpml_apply_f64(double* target, const double* src, double* psi, int axis, int sign, int kind_e,
                        const double* bc, const double* cc, const double* kc, double cb_s, const void* const* cb_p,
                        int ny, int nz, const int* box, const int* psi_box, void* s);

// amplitude mode (aux_kernels.hip): running maxima of up to 6 components, the
// changed-cell count ADDED to *changed
int fdtd_amplitude_many_f32(const void* const* f, void* const* amp, int ncomp, int ny, int nz, const int* boxes,
                            long long amp_xs, double accuracy, unsigned int* changed, void* s);
int fdtd_amplitude_many_f64(const void* const* f, void* const* amp, int ncomp, int ny, int nz, const int* boxes,
                            long long amp_xs, double accuracy, unsigned int* changed, void* s);
}
