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
#define DRSA_ETIMEOUT (-4)   /* a cooperative kernel's cross-workgroup hand-off timed out (results NaN) */

const char* drsa_amd_last_error(void);
int drsa_amd_version(void);

/* ------------------------------------------------------------------------- *
 * DRSA optimiser (cxai/xai/drsa/drsa.py)
 * Supported: d <= 128, d % K == 0, with dk = d/K padded to DKp = next power of two (<= 64)
 * and DP = next power of two >= max(16, K*DKp) <= 128.  d in {16,32,64,128} runs unpadded;
 * e.g. d = 100, K = 4 (VGGish layer 19, getdrsadata.py:119) runs as DP = 128, DKp = 32.
 * ------------------------------------------------------------------------- */

/* Bytes of device workspace needed by the drsa_* calls below for N rows (0: unsupported). */
size_t drsa_amd_drsa_workspace_bytes(int64_t N, int d, int K);

/* Floats of the gradient slab gs (DP*DP + DP/DKp, padded coordinates) exchanged between
 * drsa_amd_drsa_partial and drsa_amd_drsa_finish (the all-reduce payload of a sharded run).
 * Equals d*d + K when d is a power of two >= 16 and d/K is a power of two; 0 if unsupported. */
size_t drsa_amd_drsa_slab_floats(int d, int K);

/* Local (shard) pass: gs_out[0:DP*DP] = A^T (R (.) CU) + C^T (R (.) AU) (unscaled gradient,
 * R = relu block sums broadcast over each concept block), gs_out[DP*DP : DP*DP+Kp] = S_k =
 * sum_n relu(s_nk)^2 (padded coordinates; drsa_amd_drsa_slab_floats).  Sum gs_out over
 * shards (e.g. one RCCL all-reduce), then call drsa_amd_drsa_finish with the global row count.
 * Replaces the forward+autograd half of SubspaceOptimizer.run (drsa.py:91-100). */
int drsa_amd_drsa_partial(const float* A, const float* C, int64_t N, int d, int K, const float* U,
                          float* gs_out, void* workspace, size_t workspace_bytes, void* stream);

/* f_out[0] = objective f(U) (objective_fn, drsa.py:224-238); unless objective_only,
 * U_out = polar(U + grad f(U)) (orthogonalize, drsa.py:201-221, on device).
 * iters_out (nullable, device int) receives the Newton-Schulz iteration count. */
int drsa_amd_drsa_finish(const float* gs, int64_t N_total, int d, int K, const float* U, float* U_out,
                         float* f_out, int objective_only, int* iters_out, void* stream);

/* One fused sharded step (row-sharded DRSA; drsa.py:84-106 split over ranks): from
 * the ALL-REDUCED slab gs of the previous partials (N_total rows over all ranks) and the U they
 * were taken at, U_out = polar(U + G diag(c)) and f(U) -> f_out[0]; then the partial of this
 * rank's N rows at U_out -> gs_out (the next all-reduce's payload; may alias gs).  Equals
 * drsa_amd_drsa_finish followed by drsa_amd_drsa_partial bit for bit, in one launch fewer.
 * Available where drsa_amd_drsa_fused_supported(d, K) returns 1 (padded d = 64, block width
 * <= 16: C3, C4); otherwise use the two-call form. */
int drsa_amd_drsa_fused_supported(int d, int K);
int drsa_amd_drsa_fused_step(const float* A, const float* C, int64_t N, int d, int K, const float* gs,
                             int64_t N_total, const float* U, float* U_out, float* f_out, float* gs_out, void* ws,
                             size_t ws_size, void* stream);

/* Counter-indexed forms for a step loop captured once in a graph and replayed (the sharded loop
 * with its RCCL all-reduce, xai/drsa/distributed.py): f(U) goes to f_traj[*counter] and the device
 * int *counter is incremented by the kernel, so every replay fills the next trajectory slot.
 * Otherwise identical to drsa_amd_drsa_fused_step / drsa_amd_drsa_finish (objective_only = 0). */
int drsa_amd_drsa_fused_step_counted(const float* A, const float* C, int64_t N, int d, int K, const float* gs,
                                     int64_t N_total, const float* U, float* U_out, float* f_traj, int* counter,
                                     float* gs_out, void* ws, size_t ws_size, void* stream);
int drsa_amd_drsa_finish_counted(const float* gs, int64_t N_total, int d, int K, const float* U, float* U_out,
                                 float* f_traj, int* counter, void* stream);

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
 * stream).  At padded size 128 (d > 64) each step's polar runs on 8 cooperating workgroups
 * that hand X over through the workspace (bit-identical to drsa_amd_drsa_finish's single
 * workgroup).  They wait on each other, so they must become resident together: work running
 * concurrently on other streams only delays them, unless it holds more than 248 CUs while itself
 * waiting on this stream.  A wait that outlives 100 ms (and 20k polls) gives up: U and f are NaN
 * from that step on, the run's later finishes skip straight to NaN, and drsa_amd_drsa_run returns
 * DRSA_ETIMEOUT (it reads the workspace's status word back, synchronising the stream, at d > 64).
 * Inside a caller's stream capture that read is skipped: check drsa_amd_drsa_coop_status after
 * the replay. */
int drsa_amd_drsa_run(const float* A, const float* C, int64_t N, int d, int K, float* U_io, float* U_tmp,
                      int steps, float* f_traj, int* counter, void* workspace, size_t workspace_bytes,
                      int use_graph, void* stream);

/* Status of the cooperative finish of the last drsa_amd_drsa_run / _run_multi on this workspace
 * (same N, d, K): *status_out = 1 if a hand-off timed out (U, f NaN), else 0 (always 0 at d <= 64).
 * Synchronises `stream`; not callable while it is being captured. */
int drsa_amd_drsa_coop_status(const void* workspace, int64_t N, int d, int K, int* status_out, void* stream);

/* Test hook: the cooperative finish's spin budget in 100 MHz ticks for launches enqueued from now on
 * (0: give up at the first poll that finds a workgroup missing, with no minimum poll count);
 * -1 restores the default (100 ms and 20k polls). */
int drsa_amd_debug_coop_spin_budget(long long ticks);

/* orthogonalize (drsa.py:201-221): U_out = V (V^T V)^{-1/2}, Newton-Schulz on device, d <= 128.
 * Stop rule (polar_ns.h): iterate X <- X (3I - X^T X)/2 from the scaled V until max|X^T X - I| is
 * below the internal tolerance (4e-7), or stop after the update that starts from d * max|X^T X - I|
 * < 1e-2 (that update provably leaves a spectral error below 0.75 e^2 (1 + e/3) < 7.6e-5, e <= d *
 * max|.|; the typical spread-out error of V = U + G is ~sqrt(d) smaller), or when fp32 rounding is
 * the floor.  So the tolerance is advisory for that last update: orthogonality of the result is the
 * bound above, gated in tests/test_drsa_gpu.py at |U^T U - I| < 2e-6 (step) and 5e-6 (d = 128
 * orthogonalize) and by the DRSA trajectories against the reference's fp64 eigh at 1e-4. */
int drsa_amd_polar(const float* V, int d, float* U_out, int* iters_out, void* stream);

/* compute_subspace_relevances (explainer.py:206-242): out[b][k] = sum_n sum_{j in block k}
 * (act[b][n] U)_j (ctx[b][n] U)_j for act, ctx [B][N][d], d <= 128, K | d.  The workspace
 * (drsa_amd_subspace_relevances_workspace_bytes) holds per-chunk partial sums. */
size_t drsa_amd_subspace_relevances_workspace_bytes(int64_t B, int64_t N, int d, int K);
int drsa_amd_subspace_relevances(const float* act, const float* ctx, int64_t B, int64_t N, int d, int K,
                                 const float* U, float* out, void* workspace, size_t workspace_bytes, void* stream);


/* ------------------------------------------------------------------------- *
 * LRP engine (zennit 0.5.1 rules over the VGG-type CNN; cxai/xai/explain).
 * Enumerations shared by the calls below:
 *   xmode: 0 = R = acc, 1 = R = x * acc, 2 = R = max(x,0)*acc0 + min(x,0)*acc1
 *   post : 0 = none, 1 = g = [x > 0] R / stab(den, eps), 2 = g = [x > 0] R
 * stab(t, eps) = t + eps * (sign(t) + [t == 0])   (zennit Stabilizer)
 * ------------------------------------------------------------------------- */

/* Floats of a prepared conv weight tensor [ng][9 * cin_p][cout_p]. */
size_t drsa_amd_conv_weight_floats(int cin, int cout, int ng);

/* Forward conv3x3 'same' + bias + ReLU [+ max-pool with argmax] and the layer's LRP
 * denominator (Gamma: ng = 2 for x >= 0, where set 1 is applied to x as is, or ng = 3 with
 * the x+ / x- split; den = (z1 + bias[1]) + (z2 + bias[2]), and zennit 0.5.1's Gamma passes
 * bias[2] = 0 because its x- terms' modifiers zero the bias; Epsilon: ng = 1; WSquare/Flat: den_map).
 * pool: 0 = none (out and out_den at full resolution), 1 = 2x2, 2 = 2x4 (VGGish's (2,4) pool,
 * create_model.py:61); pooled: out = window max, out_amax = row-major index of its first
 * maximum (NaN wins, torch max_pool2d), out_den = the denominator at that pixel.
 * Replaces the model forward (create_model.py:91-97) plus the modified forwards zennit's
 * BasicHook re-runs in backward (attribute.py:98-107 via zennit.core.BasicHook).
 * Like every conv entry point below, it needs one sample's channels x H x W < 2^31 (the kernels
 * address a sample's planes with 32-bit offsets); otherwise it returns an error. */
int drsa_amd_conv_fwd(const float* in, const float* wts, const float* bias, const float* den_map, float* out,
                      uint8_t* out_amax, float* out_den, int B, int cin, int cout, int H, int W, int ng,
                      int pool, void* stream);

/* bf16-operand variant of drsa_amd_conv_fwd (the bf16 CNN with fp32 accumulate; the
 * reference has no bf16 path).  The conv input is rounded to bf16 (nearest even) as it is staged,
 * the weights come pre-rounded in the layout [ng][cin_p/16][9 taps][2][cout_p][8] bf16
 * (cin_p = pad32(cin), cout_p = pad32(cout); input channel = 16 chunk + 8 half + j, tap = 3 ky + kx;
 * drsa_amd_conv_weight_bf16_elems elements, 16-byte aligned), products are summed in fp32 on
 * v_mfma_f32_32x32x16_bf16 and everything after the accumulator (bias, ReLU, pool, argmax,
 * denominators) and every output is fp32, exactly as drsa_amd_conv_fwd.  cin > 1 only (the
 * Cin = 1 first layer stays on the fp32 kernel). */
size_t drsa_amd_conv_weight_bf16_elems(int cin, int cout, int ng);

/* 1 if drsa_amd_conv_fwd (bf16 = 0) / drsa_amd_conv_fwd_bf16 (bf16 = 1) has a kernel for this
 * shape and pool mode, else 0 (callers then pool with drsa_amd_maxpool_capture). */
int drsa_amd_conv_fwd_has_kernel(int cin, int cout, int W, int ng, int pool, int bf16);
int drsa_amd_conv_fwd_bf16(const float* in, const uint16_t* wts, const float* bias, const float* den_map, float* out,
                           uint8_t* out_amax, float* out_den, int B, int cin, int cout, int H, int W, int ng,
                           int pool, void* stream);

/* Rule backward of one conv as a transposed conv (flipped/transposed weights), with the
 * max-pool/ReLU backward folded into the input (g_amax != NULL: g at pool resolution) and
 * the next layer's division folded into the output (post).  Bq rows = samples * clones.
 * Replaces zennit's Gamma / Epsilon / WSquare / Flat gradient_mapper + reducer
 * (constants.py:27-51 rule maps). */
int drsa_amd_conv_bwd(const float* g, const uint8_t* g_amax, const float* wts, const float* x, const float* den,
                      float* out, int Bq, int clones, int cin, int cout, int H, int W, int ng, int xmode,
                      int post, float eps, void* stream);

/* bf16-operand variant of drsa_amd_conv_bwd (SURVEY C5 "VGGish-depth CNN bf16": the relevance
 * backward of a bf16 plan; the reference has no bf16 path).  g (the quotient R / stab(den) entering
 * the transposed conv, after the pool backward) is rounded to bf16 (nearest even) as it is staged,
 * the weights come pre-rounded in the forward bf16 layout of the backward weight set:
 * [cin_p/16][9 taps][2][cout_p][8] bf16 with cin = g channels (the forward cout), cout = output
 * channels (the forward cin), both padded to 32 (drsa_amd_conv_weight_bf16_elems(cin, cout, 1)
 * elements, 16-byte aligned); products are summed in fp32 on v_mfma_f32_32x32x16_bf16 and the
 * epilogue (x-multiply, the next layer's division) is fp32 as in drsa_amd_conv_bwd.  ng = 1 and
 * cin >= 16 only (the first layer keeps the fp32 kernel).  Replaces the same zennit rule
 * backward as drsa_amd_conv_bwd (constants.py:27-51). */
int drsa_amd_conv_bwd_bf16(const float* g, const uint8_t* g_amax, const uint16_t* wts, const float* x, const float* den,
                           float* out, int Bq, int clones, int cin, int cout, int H, int W, int ng, int xmode,
                           int post, float eps, void* stream);

/* drsa_amd_conv_bwd_bf16 with g at 2 x pool_w max-pool resolution (pool_w = 4: the VGGish (2,4)
 * pool of block 1, create_model.py:61; pool_w = 2 is drsa_amd_conv_bwd_bf16 with g_amax): the pool
 * backward is folded into the staging (each halo pixel takes its cell's g where the cell's argmax
 * byte, row * pool_w + col, names it), so no unpooled g is written or read.  ng = 1. */
int drsa_amd_conv_bwd_has_kernel_bf16_pw(int cin, int cout, int W, int pool_w);
/* 1 when the fp32 backward (drsa_amd_conv_bwd_den_map with g_amax) has a kernel for g at 2 x pool_w
 * pool resolution: the (2,4) pool backward folded into the fp32 staging (VGGish block 1; 2 x 4 cells
 * expanded to their 8 pixels at the LDS store; needs W / 4 % 4 == 0), bit-identical to the unpool
 * followed by the dense-g backward (the same MFMA operands). */
int drsa_amd_conv_bwd_has_kernel_pw(int cin, int cout, int W, int ng, int pool_w);
int drsa_amd_conv_bwd_bf16_pw(const float* g, const uint8_t* g_amax, int pool_w, const uint16_t* wts, const float* x,
                              const float* den, float* out, int Bq, int clones, int cin, int cout, int H, int W,
                              int xmode, int post, float eps, void* stream);

/* The backward conv (fp32 weights: wts_bf16 = 0, ng 1..2, g dense or 2x2-pool-sparse; bf16 weights:
 * wts_bf16 = 1, ng = 1, g dense or 2 x pool_w pool-sparse) with post = POST_DIV whose denominator is
 * the next layer's input-independent WSquare / Flat map den_map [cout][H][W] itself, the same plane
 * for every sample: the layer below is a WSquare / Flat conv NOT followed by a pool (VGGish block 1,
 * block_depth 2: conv0 -> conv3), so its per-sample denominator is the map and no per-sample copy
 * is written or read.  Bit-identical to drsa_amd_conv_bwd{,_bf16,_bf16_pw}(post = POST_DIV) on the
 * copy (replaces the same rule backward, attribute.py:98-107). */
int drsa_amd_conv_bwd_den_map(const float* g, const uint8_t* g_amax, int pool_w, const void* wts, int wts_bf16,
                              const float* x, const float* den_map, float* out, int Bq, int clones, int cin, int cout,
                              int H, int W, int ng, int xmode, float eps, void* stream);

/* WSquare / Flat first layer under a 2x2 max-pool, with its denominator map split for the next
 * backward (zennit WSquare/Flat: den = conv(1; W^2, b^2); constants.py:29 puts
 * WSquare on the first layer).  Such a map holds one value per channel on every pixel off its
 * 1-pixel border ring (each interior pixel sums all 9 taps in the same order), so the denominator
 * at the pool argmax is that value everywhere except near the image border.
 *   drsa_amd_conv_fwd_den_ring: drsa_amd_conv_fwd for cin = 1, pool = 1 and the map den, except
 *       that the per-sample copy of the denominator at the argmax goes only to den_ring, the border
 *       ring of float4 groups stored compactly: per (sample, channel) plane R = 2 W/2 + 8 (H/2 - 2)
 *       floats = [pooled row 0 | pooled row H/2-1 | rows 1..H/2-2 x (columns 0..3, W/2-4..W/2-1)]
 *       (H >= 4, W % 16 == 0).
 *   drsa_amd_conv_bwd_den_ring: drsa_amd_conv_bwd (wts_bf16 = 0) or _bf16 (wts_bf16 = 1) with
 *       post = POST_DIV whose denominator is den_ring (the compact ring above) on the ring and den_const4[c][0..3] (the
 *       map's interior value of channel c, 4 copies, 16-byte aligned) elsewhere.  Here H, W are the
 *       pooled resolution.
 * Together they give bit for bit what drsa_amd_conv_fwd (with out_den) + drsa_amd_conv_bwd(POST_DIV)
 * give, while only ~1/16 of the per-sample denominator copy is ever stored and read, in full
 * coalesced float4s (replace the same rule passes, attribute.py:98-107). */
int drsa_amd_conv_fwd_den_ring(const float* in, const float* wts, const float* bias, const float* den_map, float* out,
                               uint8_t* out_amax, float* den_ring, int B, int cout, int H, int W, int ng,
                               void* stream);
int drsa_amd_conv_bwd_den_ring(const float* g, const uint8_t* g_amax, const void* wts, int wts_bf16, const float* x,
                               const float* den_ring, const float* den_const4, float* out, int Bq, int clones, int cin,
                               int cout, int H, int W, int ng, int xmode, float eps, void* stream);
/* 1 if drsa_amd_conv_bwd_bf16 has a kernel for this shape (sparse: g at 2x2-pool resolution). */
int drsa_amd_conv_bwd_has_kernel_bf16(int cin, int cout, int W, int ng, int sparse);

/* Dense layer forward: z = x W^T + b [, relu(z)]  (classifier Linear layers). */
int drsa_amd_linear_fwd(const float* x, const float* W, const float* bias, float* z_out, float* relu_out, int M,
                        int N, int K, void* stream);

/* Dense layer rule backward: g = [z>0?] (R | seed) / stab(z, eps)  ->  out = epi(g W).
 * seed_cls (device int per row) replaces lrp_output_modifier (attribute.py:111-160):
 * R = one_hot ? onehot(cls) : z * onehot(cls). */
int drsa_amd_linear_bwd(const float* R, const int* seed_cls, int one_hot, const float* z, int relu_mask, int rule_eps,
                        float eps, const float* W, const float* x, int xmode, const float* den, int post,
                        float eps_post, float* out, int M, int Nout, int Kin, void* stream);

/* Projection residual P = U U^T - I (d x d, d <= 128): each entry a float64 fma chain over k
 * ascending minus the identity, rounded once to fp32 (symmetric bit for bit).  Computed once per
 * U (plan preparation); the projection calls below evaluate a' = h U^T as a + a P, so that a' at
 * dead ReLU channels is exact to its rounding. */
int drsa_amd_projection_residual(const float* U, int d, float* P, void* stream);

/* ProjectionModel forward (modify_model.py:75-123): h = a_vec U, a' = h U^T (as a + a P, P from
 * drsa_amd_projection_residual) [, 2x2 pool].
 * h and ap may be NULL (not stored); ap is required when pool == 0 (it is the output).
 * Any D <= 128 (VGGish layer 19: D = 100): zero-padded embedding in the kernel; for D % 4 == 0
 * every value is the unpadded D-term chain. */
int drsa_amd_projection_fwd(const float* a, const float* U, const float* P, float* h, float* ap, float* pooled,
                            uint8_t* amax, int B, int D, int H, int W, int pool, void* stream);

/* Epsilon(invprojection) -> SubspaceHook mask -> Epsilon(projection) -> ReLU backward ->
 * division of the conv rule below (explainer.py:198-203, attribute.py:42-60).
 * fanout == 1: each sample yields K+1 clones (standard + K subspaces); fanout == 2: the K subspace
 * clones only (the standard heatmap is then their sum, drsa_amd_heatmap_sort std_from_sum);
 * fanout == 0: row b is clone (b mod (K+1)) of a replicated batch (explainer.py:92 semantics).
 * ap or h NULL: h and a' are recomputed from a in the kernel (same MFMA order as
 * drsa_amd_projection_fwd, so the result is bit-identical to passing the stored buffers); P is
 * then required. */
int drsa_amd_projection_bwd(const float* gp, const uint8_t* amax, const float* ap, const float* h, const float* a,
                            const float* den, const float* U, const float* P, float* G, int B, int D, int H, int W,
                            int K, float eps_proj, float eps_den, int fanout, void* stream);

/* AlphaBeta on a conv with non-negative input (zennit AlphaBeta as configured at pf.py:285-289,
 * restated in oracle/lrp_ref.py): split R at the conv output into gp = R / stab(den_p) and
 * gn = R / stab(den_n) (den per sample, R rows = sample*clones + clone, n elements per row) ... */
int drsa_amd_ab_split(const float* g, const float* den_p, const float* den_n, float* gp, float* gn, int Bq,
                      int clones, int64_t n, float eps, void* stream);
/* ... and after the two backward convs pos = x J^T_{W+} gp, neg = x J^T_{W-} gn:
 * R_in = alpha*pos - beta*neg, then the post step of the layer below (post as conv_bwd). */
int drsa_amd_ab_combine(const float* pos, const float* neg, float alpha, float beta, const float* x, const float* den,
                        float* out, int Bq, int clones, int64_t n, int post, float eps, void* stream);

/* First-layer (one input channel) WSquare / Flat backward: R = J^T_{W2} g. */
int drsa_amd_first_layer_bwd(const float* g, const uint8_t* amax, const float* w2, float* out, int Bq, int clones,
                             int C, int H, int W, void* stream);

/* Input-independent WSquare / Flat denominator map conv(1; W2, b2): [C][H][W]. */
int drsa_amd_first_layer_den(const float* w2, const float* b2, float* den, int C, int CI, int H, int W, void* stream);

/* HeatmapGenerator post-processing (explainer.py:99-123, sort_subspaces 151-176): standard
 * heatmap + relevance, subspace heatmaps sorted by descending relevance, relevances, mask
 * (int64, numpy argsort(...)[..., ::-1] order; relevances are numpy's float32 sums).
 * std_from_sum = 0: hm is [B][K+1][HW] with the standard heatmap first (clone 0);
 * std_from_sum = 1: hm is [B][K][HW] (concept maps only) and the standard heatmap is their sum,
 * k ascending (equal to clone 0 in exact arithmetic: every LRP rule is linear in the relevance). */
int drsa_amd_heatmap_sort(const float* hm, int B, int K, int HW, int std_from_sum, float* std_out, float* std_rel,
                          float* sub_out, float* rel, int64_t* mask, void* stream);

/* One DRSA problem for drsa_amd_drsa_run_multi (all pointers device memory; the fields mean what
 * the same-named arguments of drsa_amd_drsa_run mean). */
typedef struct drsa_amd_problem {
  const float* A;
  const float* C;
  int64_t N;
  int d;
  int K;
  float* U_io;
  float* U_tmp;
  float* f_traj; /* [steps + 1] */
  int* counter;
  void* ws;
  size_t ws_size;
  int dtype; /* 0: A, C fp32; 1 / 2: A, C bf16 / fp16 (uint16 bit patterns), GEMM1 on bf16 / fp16
              * MFMA with fp32 accumulation, padded d >= 32 */
} drsa_amd_problem_t;

/* drsa_amd_drsa_partial with A, C stored as bf16 (C5: bf16 input; the U-projection GEMM runs on
 * bf16 MFMA with fp32 accumulation, U rounded to bf16 per step; the gradient GEMM and every
 * reduction stay fp32).  No reference bf16 path exists: its tolerance is looser (tests). */
int drsa_amd_drsa_partial_bf16(const uint16_t* A, const uint16_t* C, int64_t N, int d, int K, const float* U,
                               float* gs_out, void* ws, size_t ws_size, void* stream);
/* The same with A, C as fp16 (C5's "fp16 MFMA projection": v_mfma_f32_16x16x32_f16, U rounded to
 * fp16 once per launch, fp32 accumulate; everything after GEMM1 fp32). */
int drsa_amd_drsa_partial_f16(const uint16_t* A, const uint16_t* C, int64_t N, int d, int K, const float* U,
                              float* gs_out, void* ws, size_t ws_size, void* stream);

/* P independent problems advanced S steps together (C5: two layers, K=16 each, one graph).
 * Replaces the sequential per-layer loop of optsubspaces.py:18-23 / drsa.main. */
/* Returns DRSA_ETIMEOUT like drsa_amd_drsa_run when a problem's cooperative finish timed out.
 * Capturable: inside a caller's stream capture it records the per-problem chains on forked side
 * streams (a per-thread pool that outlives the call) joined back into `stream`, and skips its own
 * graph and the status read-back (drsa_amd_drsa_coop_status per problem after the replay). */
int drsa_amd_drsa_run_multi(int P, const drsa_amd_problem_t* probs, int steps, int use_graph, void* stream);

/* P independent fp32 problems sharing one padded geometry (same pow2(d) and concept width; N may
 * differ) advanced together with ONE launch per phase for all of them: every problem's partial
 * on about `blocks` workgroups (0: about sixteen waves of workgroups over the chip), each owning whole
 * groups of the fixed 256-leaf row partition that drsa_amd_drsa_run uses, the slab reduces, then
 * every problem's finish on its own workgroup.  The task-parallel DRSA grid of the reference's
 * cluster driver (optsubspaces.py:17-23: classes x layers x runs, each drsa.main(..., steps=5000)).
 * Fields of probs mean what they mean for drsa_amd_drsa_run_multi (dtype must be 0).  Every
 * problem's trajectory and U equal drsa_amd_drsa_run's bit for bit, for any `blocks`.  Not stream-
 * capturable (it allocates its descriptor table); synchronises the stream before returning. */
int drsa_amd_drsa_run_batched(int P, const drsa_amd_problem_t* probs, int steps, int blocks, int use_graph,
                              void* stream);

/* ------------------------------------------------------------------------- *
 * Log-mel front end
 * Replaces cxai/utils/dataloading.py:62-74 + :138-176 (Loader: torchaudio
 * Spectrogram(n_fft, hop, power=None) -> MelScale(n_mels) -> log10(+log_eps) -> clamp ->
 * frames [frame0, frame0+width)) fused with cxai/utils/sound.py:8-44 (get_slice chunking)
 * and :67-70 (peak_normalizer).
 *   wav: songs [n_songs] at stride song_stride floats; chunk c of a song starts at
 *        c*chunk_hop and is chunk_len samples long (get_slice's unfold).
 *   window: [n_fft] analysis window (torch.hann_window(n_fft), periodic).
 *   band_*: the mel filterbank [n_fft/2+1, n_mels] in band form: filter m covers FFT bins
 *        band_lo[m] .. band_lo[m]+band_n[m]-1 with weights band_w[band_off[m] ...].
 *   peak_norm: divide each chunk by its max |x| (peak_normalizer).
 *   out: [n_songs*chunks_per_song, n_mels, width] fp32.
 * Needs n_fft/2 = 2^a 3^b 5^c; LDS footprint (drsa_amd_logmel_smem_bytes) <= 160 KB.
 * ------------------------------------------------------------------------- */
int drsa_amd_logmel_smem_bytes(int n_fft, int hop, int n_mels, int width, int band_nnz);
int drsa_amd_logmel(const float* wav, int64_t n_songs, int64_t song_stride, int chunks_per_song, int64_t chunk_hop,
                    int chunk_len, int n_fft, int hop, int n_mels, int width, int frame0, const float* window,
                    const int* band_lo, const int* band_n, const int* band_off, const float* band_w, int band_nnz,
                    int peak_norm, int clamp, float clamp_min, float log_eps, float* out, void* stream);

/* ------------------------------------------------------------------------- *
 * DRSA training data: cxai/xai/drsa/preprocessing.py:18-256 and
 * cxai/xai/drsa/cluster/getdrsadata.py:47-59.
 * ------------------------------------------------------------------------- */

/* ph x pw max-pool (stride = kernel) of a full-resolution ReLU output with the engine's argmax
 * byte (dy*pw + dx of the first maximum) and the rule denominator gathered at the argmax (den
 * may be NULL).  Keeps the layer-j activation map for DRSA data (the reference's store_hook,
 * preprocessing.py:92-103) and runs the pools the fused conv epilogue does not (VGGish (2,4),
 * create_model.py:61 pool_kernels). */
int drsa_amd_maxpool_capture(const float* a, const float* den, float* y, uint8_t* amax, float* den_pooled, int B,
                             int C, int H, int W, int ph, int pw, void* stream);

/* Full-resolution map from its pooled form + argmax (ph x pw pool): layer.output.grad of
 * get_intermediate (preprocessing.py:156-158), and the max-pool backward of pools other than
 * 2x2.  rel rows are sample*clones + clone, amax rows are samples.  out [Bq, C, H, W]. */
int drsa_amd_relevance_unpool(const float* rel, const uint8_t* amax, int Bq, int clones, int C, int H, int W, int ph,
                              int pw, float* out, void* stream);

/* Activation vectors and context vectors C = R / (A + 1e-7) at sampled locations
 * (get_vectors_from_maps + compute_context_vectors, preprocessing.py:179-193, 234-256).
 *   act [B, C, H, W]; rel full [B, C, H, W] (rel_amax NULL) or pooled [B, C, H/ph, W/pw] + argmax.
 *   idx [B, L] int32 flat locations (sample_spatial_locations), or NULL = every location
 *   (L = H*W, inference branch, [B, H*W, C]).
 *   layout 0 = the reference's get_vectors_from_maps row order (transpose-then-reshape),
 *   layout 1 = one row per (sample, location).  A_out, C_out [B*L, C]. */
int drsa_amd_drsa_vectors(const float* act, const float* rel, const uint8_t* rel_amax, const int* idx, int B, int C,
                          int H, int W, int ph, int pw, int L, int layout, float* A_out, float* C_out, void* stream);

/* normalize_vectors (preprocessing.py:219-231): out = v / sqrt(mean(v^2)) / d^(1/4) over all
 * n elements (deterministic fp64 reduction).  out may alias v. */
size_t drsa_amd_normalize_workspace_bytes(void);
int drsa_amd_normalize_vectors(const float* v, int64_t n, int d, float* out, void* ws, size_t ws_bytes, void* stream);

/* The same normalisation over rows spread across ranks (getdrsadata.py:47-59 normalises the whole
 * 1000-sample x 20-location set at once, preprocessing.py:229-231):
 *   drsa_amd_normalize_sumsq: this rank's sum of v^2 -> sum_out[0] (fp64, device; the fixed-order
 *       reduction of drsa_amd_normalize_vectors; 0 for n == 0);
 *   drsa_amd_normalize_scale: E = sqrt((sums[0] + ... + sums[nsums-1], in that order) / n_total),
 *       out = v / E / d^(1/4) over this rank's n elements.  sums are the ranks' sum_out values in
 *       rank order (one all-gather), n_total the element count over all ranks.  out may alias v.
 * With nsums = 1 and n_total = n this is drsa_amd_normalize_vectors up to the fp64 sum's last bit. */
int drsa_amd_normalize_sumsq(const float* v, int64_t n, void* ws, size_t ws_bytes, double* sum_out, void* stream);
int drsa_amd_normalize_scale(const float* v, int64_t n, int d, const double* sums, int nsums, int64_t n_total,
                             float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DRSA_AMD_H */
