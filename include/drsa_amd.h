/*
 * drsa_amd — C ABI of the MI355X (gfx950) DRSA audio-explanation engine.
 *
 * Plain pointers and sizes only; every pointer argument is a DEVICE pointer unless
 * stated otherwise; `stream` is a hipStream_t (NULL = legacy default stream).
 * Every entry point returns 0 on success, a negative DRSA_E* code on an argument
 * error, or a positive hipError_t; it never throws.  drsa_amd_last_error() gives the
 * message of the last failure on the calling thread.
 *
 * Layouts: activations/relevances NCHW fp32 (the reference's torch layout);
 * A, C row-major [N, d] fp32; U row-major [d, d] fp32.
 *
 * Each entry point names the reference interface it replaces (file:line in
 * sharckhai/drsa-audio @ 2024-12-20, paths relative to the repository root).
 */
#ifndef DRSA_AMD_H
#define DRSA_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRSA_OK 0
#define DRSA_EINVAL (-1)
#define DRSA_EWORKSPACE (-2)
#define DRSA_EUNSUPPORTED (-3)

const char* drsa_amd_last_error(void);
int drsa_amd_version(void);

/* ------------------------------------------------------------------------- *
 * DRSA optimiser (cxai/xai/drsa/drsa.py)
 * Supported: d in {16, 32, 64, 128}; d % K == 0; d/K in {1,2,4,8,16,32,64}.
 * ------------------------------------------------------------------------- */

/* Bytes of device workspace needed by the drsa_* calls below for N rows. */
size_t drsa_amd_drsa_workspace_bytes(int64_t N, int d, int K);

/* Local (shard) pass: gs_out[0:d*d] = A^T (R (.) CU) + C^T (R (.) AU) (unscaled gradient,
 * R = relu block sums broadcast over each concept block), gs_out[d*d : d*d+K] = S_k =
 * sum_n relu(s_nk)^2.  Sum gs_out over shards (e.g. one RCCL all-reduce), then call
 * drsa_amd_drsa_finish with the global row count.
 * Replaces the forward+autograd half of SubspaceOptimizer.run (drsa.py:91-100). */
int drsa_amd_drsa_partial(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                          float* gs_out, void* workspace, size_t workspace_bytes, void* stream);

/* f_out[0] = objective f(U) (objective_fn, drsa.py:224-238); unless objective_only,
 * U_out = polar(U + grad f(U)) (orthogonalize, drsa.py:201-221, on device).
 * iters_out (nullable, device int) receives the Newton-Schulz iteration count. */
int drsa_amd_drsa_finish(const float* gs, int64_t N_total, int d, int K, const float* U, float* U_out,
                         float* f_out, int objective_only, int* iters_out, void* stream);

/* One SubspaceOptimizer.run iteration (drsa.py:84-106): f_out[0] = f(U), U_out = new U. */
int drsa_amd_drsa_step(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                       float* U_out, float* f_out, void* workspace, size_t workspace_bytes, void* stream);

/* SubspaceOptimizer.obj_val + objective_fn (drsa.py:122-155): f_out[0] = f(U). */
int drsa_amd_drsa_objective(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                            float* f_out, void* workspace, size_t workspace_bytes, void* stream);

/* SubspaceOptimizer.run(steps) (drsa.py:76-117) without file output: f_traj[0..steps]
 * (steps+1 floats) receives the objective before every update and after the last;
 * U_io holds U_0 on entry and U_steps on exit; U_tmp is d*d scratch; counter is one
 * device int.  use_graph != 0 replays a captured two-step hipGraph (needs a non-NULL
 * stream). */
int drsa_amd_drsa_run(const float* A, const float* C, int64_t N, int d, int K, float* U_io, float* U_tmp,
                      int steps, float* f_traj, int* counter, void* workspace, size_t workspace_bytes,
                      int use_graph, void* stream);

/* orthogonalize (drsa.py:201-221): U_out = V (V^T V)^{-1/2}, Newton-Schulz on device. */
int drsa_amd_polar(const float* V, int d, float* U_out, int* iters_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DRSA_AMD_H */
