/*
 * stein_thinning_hip.h -- C ABI of the MI355X (gfx950) Stein-thinning engine.
 *
 * Drop-in boundary for the hot path of the reference's third-party dependency `stein_thinning`
 * (imported at code/src/thinning.py:5, code/src/utils/ksd.py:5-6, code/tests/test_ksd.py:3 of
 * aglebov/gradient-free-mcmc-postprocessing).  The Python shim package `stein_thinning`
 * (gradient-free-mcmc-postprocessing_amd/stein_thinning) binds these symbols with ctypes; see
 * INTEGRATION.md for the binding a maintainer adds.
 *
 * Conventions (all functions):
 *   - plain C types only; device pointers are HIP device memory owned by the caller;
 *   - `stream` is a hipStream_t (NULL = default stream); every function is asynchronous on it,
 *     allocates nothing and never synchronises (graph-capturable) -- except the one-time
 *     multi-GPU setup calls st_mailbox_alloc / st_mailbox_free / st_ipc_*, which are synchronous;
 *   - sample / gradient arrays are SoA: element (i, k) of the (n, d) array lives at p[k * ld + i],
 *     ld a multiple of 8 and >= n (the ABI's requirement, checked; the Python shim pads to a
 *     multiple of 64, one wave's rows, which the kernels do not require); per-row arrays (weights, running sums) have ld entries (rows
 *     n..ld-1 are padding: read, and in the running sums overwritten, never selected);
 *     all device pointers 16-byte aligned;
 *   - the preconditioner is isotropic Gamma^-1 = linv_scale * I ('id', 'med', 'sclmed', float
 *     options of the reference); linv_trace = np.trace(Gamma^-1) computed on the host;
 *   - weights == NULL selects the Langevin Stein kernel k_P; weights = w = exp(log q - log p)
 *     (anchored) selects the gradient-free kernel k_PQ(i,j) = w_i w_j k_Q(i,j) (report.tex:390-400);
 *   - return value: ST_OK (0) or a negative ST_ERR_*; st_last_error() describes the last failure
 *     of the calling thread.  No C++ exception crosses the ABI.
 */
#ifndef STEIN_THINNING_HIP_H
#define STEIN_THINNING_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ST_ABI_VERSION 1

#define ST_OK 0
#define ST_ERR_INVALID (-1)     /* bad argument: sizes, null pointers, alignment */
#define ST_ERR_UNSUPPORTED (-2) /* e.g. d > 128 */
#define ST_ERR_HIP (-3)         /* HIP runtime error (launch / memset) */

int st_abi_version(void);
const char *st_last_error(void);

/* ------------------------------------------------------------------------------------------
 * Greedy selection -- replaces stein_thinning.thinning._greedy_search(n_points, integrand)
 * (restated at code/notebooks/examples/JAX_Stein_Thinning.ipynb cell 22, json lines ~281-295;
 * Algorithm 3, report/report.tex:413-426) for the integrands built by _make_stein_integrand /
 * _make_stein_gf_integrand (called at code/src/utils/ksd.py:25, Gaussian_mixture.ipynb cell 93).
 * ---------------------------------------------------------------------------------------- */

/* bytes of device workspace st_greedy / st_greedy_steps / st_greedy_step need (no zeroing needed) */
int64_t st_greedy_workspace_bytes(int64_t n, int32_t d, int32_t nranks);

/*
 * Kernel-variant tuning (process-wide, host side; for measurement sweeps -- defaults are the
 * measured best on MI355X): key 0 = grid cap (blocks, 1..1024), key 1 = candidates per lane
 * (1, 2, 4; d = 2 and 4 kernels; -1 = automatic), key 2 = register prefetch of the next tile
 * (0/1; -1 = automatic), key 3 = persistent kernel register rows per thread (4, 8 on 512-thread blocks;
 * 1, 2, 4 on 256-thread blocks; -1 = automatic: 1 / 2 for blocks of at most 256 / 512 rows, 4 on other
 * 256-thread blocks, 8 on 512-thread blocks unless that leaves slots empty, then 4; 0 = disable the
 * persistent kernel; round 6 pruned the plans that won nothing), key 4 = persistent kernel threads per
 * block (256, 512; -1 = automatic: 512 with dynamic chunks above 1280 rows per block), key 5 = persistent kernel grid cap (blocks per device,
 * 1..256; -1 = one per CU), key 6 = grid cap of the d > 8 step kernel (1..1024), key 7 = proxy
 * kernel (0 = automatic: matrix cores for 16 < d <= 64; 1 = always the VALU kernel), key 8 =
 * persistent kernel blocks per CU (1 / -1 only: the two-block plans were pruned in round 6), key 9 = persistent kernel
 * record pitch in bytes (power of two, 16..4096; -1 = automatic = 256 with one replica, 16 with
 * several, narrowed to what the workspace holds), key 10 = persistent kernel record replicas
 * (power of two, 1..32: every block stores its per-step record into each replica and block b
 * sweeps replica b % replicas; -1 = automatic), key 11 = arithmetic of the d <= 8 greedy kernels
 * (1 = compact, the default: the kernel value regrouped around one reciprocal square root, a few
 * ulps from NumPy's evaluation, for every pair whose two rows and l, tr lie in [2^-60, 2^60];
 * 0 = exact: NumPy's evaluation order rounding for rounding; other pairs are always exact -- see
 * oracle/stein_ref.c and DESIGN.md §3; all ranks of a sharded run must use the same value), key 12 =
 * register rows per thread of the one-device compact-only persistent kernel, used from 8 x 512 rows per
 * block (8, 9; 0 = do not use it; -1 = automatic: 9, or 8 under the near-tie guard), key 13 = energy-distance kernel variant (0 / -1 = automatic = 1:
 * one partial sum per thread, 4 blocks per CU; 2..5: more partial sums or 8 blocks per CU; 6: the
 * round-2 zero-distance select -- measured alternatives; same distances, sums within
 * rounding), key 14 = energy-distance work units: grid blocks (256 columns x one B chunk) that
 * st_distance_colsum_ws aims for (256 .. 2^22; -1 = automatic = 32768; the B range is split into
 * that many / ceil(na / 256) chunks of at least 1024 points -- sums within rounding), key 15 = the
 * 512-thread persistent kernels keep the streamed rows' running sums in LDS (1) instead of HBM (0;
 * -1 = automatic: 1 under the near-tie guard, whose rescans read them every step, else 0 -- measured
 * slower there; same results), key 16 = persistent kernels:
 * ticks of the 100 MHz s_memrealtime clock added to a step's first winner poll before it is aligned
 * to the chip-wide poll grid (0 .. 450; -1 = automatic = 10 for the one-device compact-only kernel,
 * 0 otherwise;
 * timing only, same results), key 17 = LV gradient phase B: 1 reads the observation times / data
 * from global memory as round 3 did (0 / -1 = automatic: staged in LDS when 3 t_n doubles fit
 * 64 KB; same results), key 18 = LV gradient phase B: observation pieces per lane (1, 2, 3; -1 =
 * automatic; the per-point sum is reassociated differently, within the 1e-8 tolerance), key 19 =
 * 512-thread persistent kernels: two LDS-row chunks computed as two independent chains (1 / -1 =
 * automatic) or one after the other (0; same results), key 20 = near-tie guard of the compact
 * arithmetic (1 / -1 = on, the default; 0 = off; see st_greedy_near_tie; same indices and sums), key 22 = key 11 for the
 * launches of the CALLING HOST THREAD only (-1 = none: key 11 applies; 0 / 1 as key 11) -- the library keeps
 * it per thread, so threads thinning side by side (one per GPU) never change each other's arithmetic, key
 * 23 = key 5 for the calling host thread only (-1 = none; 1..512 blocks).
 */
int st_tune(int32_t key, int32_t value);

/* the current value of a greedy-kernel st_tune key (0 .. 6, 8 .. 12, 15, 16, 19, 20, 22, 23; -1 = automatic);
 * INT32_MIN for other keys (save / restore around a temporary setting) */
int32_t st_tune_get(int32_t key);

/* doubles per rank-candidate record {value, global index bits, x[d], g[d], w} (even) */
int64_t st_candidate_stride(int32_t d);

/*
 * Whole greedy run on one device: idx_out[0..n_points) (device, uint32) receives the selected
 * row indices exactly as the reference's `thin` / `thin_gf` / `_greedy_search` return them;
 * a_work (ld doubles, device) ends holding the running sums A after the last step.
 * For d = 2 and 4 the run is ONE launch of the persistent on-chip-resident kernel (grid checked
 * against the occupancy query first)
 * (one block per CU; rows held in VGPRs/LDS across steps); if its internal bounded wait times
 * out, the unwritten entries of idx_out are set to UINT32_MAX (callers check idx < n).
 * Other d: one fused launch per step.
 */
int st_greedy(const double *x_soa, const double *g_soa, const double *weights, int64_t n,
              int32_t d, int64_t ld, double linv_scale, double linv_trace, int64_t n_points,
              uint32_t *idx_out, double *a_work, void *workspace, int64_t workspace_bytes,
              void *stream);

/*
 * Near-tie guard of the compact arithmetic (st_tune key 20).  A guarded run (the compact arithmetic, d = 2
 * or 4; persistent kernel, batch and multi-rank included) flags the first step t whose selection the
 * arithmetic could have decided differently from the reference's NumPy evaluation: the smallest running
 * sum of any row other than the winner and the rows equal to it bit for bit (x, g, w: repeated MCMC rows,
 * adjacent or not, tie in every arithmetic and lose to the lower index on both paths) -- any other exact
 * tie included -- within thr(t) of the winner's, thr(t) a bound on how far two rows' sums may move between
 * the compact arithmetic, the exact one and NumPy's (oracle/stein_ref.c sr_greedy_mt_ties states the rule
 * and the bound; the reference's argmin is JAX_Stein_Thinning.ipynb:291-292, np.argmin of the running
 * sums).  A multi-rank run (st_greedy_sharded) flags in each rank's workspace the steps its own rows
 * flag against the global winner (bounds over all n rows): the first flagged step of the thin is the
 * minimum over the ranks (one all-reduce after the run).  Reads the workspace of a completed st_greedy /
 * st_greedy_batch / st_greedy_sharded problem after synchronising `stream` (the one exception to the
 * enqueue-only rule: a few bytes come back): *step_out = the first flagged step, -1 when none, -2 when the
 * run was not guarded (exact arithmetic, guard off, other d, or the launch-per-step kernels).  Callers
 * re-run a flagged thin with the exact arithmetic (st_tune key 11 = 0, or key 22 for the calling thread).
 */
int st_greedy_near_tie(const void *workspace, int64_t workspace_bytes, int64_t *step_out, void *stream);

/*
 * Up to 8 independent whole greedy runs of one d (2 or 4) and one n_points in ONE launch of the
 * persistent kernel: problem q gets about #CU / count blocks and runs on them exactly as st_greedy
 * would on a grid of that many blocks -- idx_out[q] and a_work[q] as st_greedy's, same indices.
 * The arrays are host arrays of count entries (device pointers / sizes per problem, as st_greedy
 * takes them); weights is NULL or has an entry for every problem.  Returns ST_ERR_UNSUPPORTED
 * (nothing enqueued) when the problems do not all plan onto the same kernel at that grid (threads
 * per block and register rows follow each problem's rows per block, as in st_greedy; e.g. a 2e5-row
 * problem next to a 2e4-row one); the caller then runs st_greedy per problem.  A timed-out
 * run poisons its own idx_out only.  Replaces the reference's loop of thin() calls over chains
 * (Stein_thinning.ipynb; code/src/utils/parallel.py:48-52 fans them out to processes).
 */
int st_greedy_batch(int32_t count, const double *const *x_soa, const double *const *g_soa,
                    const double *const *weights, const int64_t *n, int32_t d, const int64_t *ld,
                    const double *linv_scale, const double *linv_trace, int64_t n_points,
                    uint32_t *const *idx_out, double *const *a_work, void *const *workspace,
                    const int64_t *workspace_bytes, void *stream);

/*
 * Steps [t_begin, t_end) of the same single-device run (t = 0 is the diagonal); when t_end ==
 * n_points the finalize kernel writing idx_out[n_points-1] follows.  The workspace carries the
 * per-block candidate records between calls, so consecutive ranges on one stream compose into
 * st_greedy.  Used to time single step launches.
 */
int st_greedy_steps(const double *x_soa, const double *g_soa, const double *weights, int64_t n,
                    int32_t d, int64_t ld, double linv_scale, double linv_trace, int64_t t_begin,
                    int64_t t_end, int64_t n_points, uint32_t *idx_out, double *a_work,
                    void *workspace, int64_t workspace_bytes, void *stream);

/*
 * One greedy step of a row-sharded run (multi-GPU; one process per GPU).  This rank holds rows
 * [row_offset, row_offset + n) of the global sample.  Step t = 0 evaluates the diagonal; step
 * t >= 1 reads the R = nranks candidate records of step t-1 (cands_in, R * stride doubles),
 * writes idx_out[t-1] and updates the running sums.  Every step writes this rank's candidate
 * record (stride doubles) to cand_out; the caller all-gathers the records (RCCL) into the next
 * step's cands_in.
 * After the last step, st_greedy_finalize writes idx_out[n_points-1].
 */
int st_greedy_step(const double *x_soa, const double *g_soa, const double *weights, int64_t n,
                   int32_t d, int64_t ld, double linv_scale, double linv_trace,
                   int64_t row_offset, int64_t t, int32_t nranks, const double *cands_in,
                   double *cand_out, uint32_t *idx_out, double *a_work, void *workspace,
                   int64_t workspace_bytes, void *stream);

int st_greedy_finalize(const double *cands_in, int32_t nranks, int32_t d, uint32_t *idx_out,
                       int64_t t, void *stream);

/* ------------------------------------------------------------------------------------------
 * Multi-GPU greedy with device-side exchange (one process per GPU of one node, up to 8).
 * Same result as st_greedy on the whole sample (and as the reference's _greedy_search).
 *
 * Every rank holds the FULL standardised arrays (replicated, read-only: the winner's row is then
 * local) and runs ONE persistent launch over its row block [row_begin, row_end).  Per step the
 * ranks exchange their local winners {A_min, global index} through per-rank mailboxes: each rank
 * allocates one (st_mailbox_alloc: uncached device memory), exports it (st_ipc_get_handle), the
 * handles are all-gathered out of band (torch.distributed), each rank maps its peers'
 * (st_ipc_open_handle) and passes the table peer_mailboxes[0..nranks) (its own at [rank]).
 * st_mailbox_handshake verifies the round trip (ok_device[0] = 1) before the first run.
 * seq_base: exchange sequence number of this run's step 0; every rank passes the same value and
 * a following run on the same mailboxes uses seq_base + n_points.
 * Returns ST_ERR_UNSUPPORTED when d is not 2 or 4, or d = 50 with more than 256 rows per CU in
 * this rank's block (use st_greedy_step_exchange or st_greedy_step + RCCL instead); a run
 * whose peers do not answer within the kernel's bounded waits poisons idx_out (UINT32_MAX).
 * ---------------------------------------------------------------------------------------- */
int64_t st_mailbox_bytes(int32_t nranks);
int st_mailbox_alloc(int64_t bytes, void **mailbox);
int st_mailbox_free(void *mailbox);
int st_ipc_handle_bytes(void);
int st_ipc_get_handle(void *dev_ptr, void *handle_out);
int st_ipc_open_handle(const void *handle, void **dev_ptr);
int st_ipc_close_handle(void *dev_ptr);
int st_mailbox_handshake(void *const *peer_mailboxes, int32_t nranks, int32_t rank,
                         uint64_t token, int32_t *ok_device, void *stream);
int st_greedy_sharded(const double *x_soa, const double *g_soa, const double *weights, int64_t n,
                      int32_t d, int64_t ld, double linv_scale, double linv_trace,
                      int64_t row_begin, int64_t row_end, int32_t rank, int32_t nranks,
                      void *const *peer_mailboxes, uint64_t seq_base, int64_t n_points,
                      uint32_t *idx_out, double *a_work, void *workspace,
                      int64_t workspace_bytes, void *stream);
/* 1 if st_greedy_sharded would run this rank's block [row_begin, row_end) on the current device
 * (the launcher's exact decision: d, rows per block against the kernel's register/LDS budget, the
 * st_tune grid cap), 0 if it would return ST_ERR_UNSUPPORTED, < 0 on invalid arguments.  No GPU
 * work; callers agree on it across ranks before choosing the engine. */
int st_greedy_sharded_supported(int64_t n, int32_t d, int32_t has_weights, int64_t row_begin,
                                int64_t row_end, int32_t rank, int32_t nranks, int64_t n_points);
/*
 * Any d (the launch-per-step path of st_greedy_step) with the per-step rank exchange through the
 * same mailboxes instead of an RCCL all-gather: one call = the step kernel over this rank's shard
 * + a one-block exchange kernel that pushes this rank's candidate record into slot `rank` of every
 * peer's mailbox and collects the nranks records of this step into cands (nranks * stride
 * doubles; the next call's input, as st_greedy_step's cands_in).  No host synchronisation or
 * collective inside, so the m-step loop can be captured into one HIP graph and replayed; flags
 * carry a device-side exchange counter, so replays never see stale records.  All ranks must make
 * the same sequence of calls.  A peer that does not answer within the bounded wait (10 s at t = 0,
 * 2 s otherwise) sets status_device[0] = 1; later exchanges then return at once (the indices of
 * that run are garbage and the mailbox set must not be reused).  Finish with st_greedy_finalize
 * (cands, nranks).
 */
int st_greedy_step_exchange(const double *x_soa, const double *g_soa, const double *weights,
                            int64_t n, int32_t d, int64_t ld, double linv_scale, double linv_trace,
                            int64_t row_offset, int64_t t, int32_t rank, int32_t nranks,
                            void *const *peer_mailboxes, double *cands, uint32_t *idx_out,
                            double *a_work, void *workspace, int64_t workspace_bytes,
                            uint32_t *status_device, void *stream);

/* ------------------------------------------------------------------------------------------
 * Proxy producers for thin_gf -- replaces the O(n d^2) host prep of
 *   gaussian_thin (code/src/thinning.py:15-16): scipy.stats.multivariate_normal.logpdf(x, mean,
 *     cov) and -np.einsum('ij,kj->ki', np.linalg.inv(cov), x - mean)           (df = 0)
 *   thin_gf_t (Gradient_free_Student_t.ipynb cells 29, 31, 40): scipy.stats.multivariate_t.logpdf
 *     (x, loc, shape, df) and t_grad_log_pdf(x, loc, shape, df)                (df > 0)
 * x: row-major (n, d) device array (the caller's NumPy layout); loc (d); whiten (d, d) row-major =
 * scipy's _PSD(cov).U; precision (d, d) row-major = np.linalg.inv(cov); c_log = rank * log(2 pi) +
 * log_pdet (Gaussian) or A - B - C - D of scipy's multivariate_t._logpdf (t).  Writes log_q_out (n)
 * and grad_out (row-major (n, d)).  Per-row dot products are summed in a different order than
 * NumPy/BLAS (fp64 tolerance, not bit-identical).
 * ---------------------------------------------------------------------------------------- */
int st_proxy_logpdf_grad(const double *x, int64_t n, int32_t d, const double *loc,
                         const double *whiten, const double *precision, double df, double c_log,
                         double *log_q_out, double *grad_out, void *stream);

/* ------------------------------------------------------------------------------------------
 * KDE proxy -- replaces jax.scipy.stats.gaussian_kde(sample.T, bw_method, weights).logpdf and its
 * jax.grad as the reference's Gaussian-mixture study feeds them to thin_gf (Gaussian_mixture.ipynb
 * cells 42-48, 51).  Whitened data p = x L (n points, SoA (d, ldp)) and queries q = y L (m points,
 * SoA (d, ldq)), L = cholesky(KDE precision) (HOST-computed; `whiten` = L on the DEVICE, (d, d)
 * row-major); log_weights (n, device) or NULL for the uniform log_weight_uniform:
 *   log_q[j] = logsumexp_i(log w_i + log_norm - |p_i - q_j|^2 / 2),
 *   grad[j]  = (sum_i softmax_i(.) p_i - q_j) L^T   (row-major (m, d)).
 * workspace: st_kde_workspace_bytes(m, d) bytes (0 for d <= 8).
 * ---------------------------------------------------------------------------------------- */
int64_t st_kde_workspace_bytes(int64_t m, int32_t d);
int st_kde_logpdf_grad(const double *p_soa, int64_t ldp, int64_t n, const double *log_weights,
                       double log_weight_uniform, const double *q_soa, int64_t ldq, int64_t m, int32_t d,
                       double log_norm, const double *whiten, double *log_q_out, double *grad_out,
                       void *workspace, int64_t workspace_bytes, void *stream);

/* ------------------------------------------------------------------------------------------
 * Lotka-Volterra inputs, batched over n parameter points (one RK45 integration per point, scipy's
 * solve_ivp algorithm step for step -- code/src/lotka_volterra.py):
 *   st_lv_grad_log_posterior: grad_out (n, 4) row-major = grad_log_posterior(theta) of
 *     Sensitivity_analysis.ipynb cells 40, 46 (forward sensitivities, solve_ivp(
 *     lotka_volterra_sensitivity, ..., dense_output=True).sol(t));
 *   st_lv_log_target_density: out (n) = lotka_volterra.log_target_density(log_theta) (2-state
 *     system), theta = exp(log_theta) computed by the caller (NumPy's exp, as the reference).
 * theta, log_theta: (n, 4) row-major device arrays; t_eval (t_n) ascending and y_obs (t_n, 2)
 * row-major: the observation times and data (device); span_u0_tol: HOST array {t0, t1, u0_1,
 * u0_2, rtol, atol}; cov_inv: HOST (2, 2) row-major inv(C); whiten: HOST (2, 2) row-major scipy
 * _PSD(C).U with c_log = rank * log(2 pi) + log_pdet; norm_logc = log(sqrt(2 pi)) (scipy.stats.norm).
 * status (n, device): 0 ok, 1 step size fell below scipy's min_step (output NaN), 2 max_steps
 * reached (output NaN).  Results agree with scipy to rounding (BLAS summation orders differ).
 * ---------------------------------------------------------------------------------------- */
int st_lv_grad_log_posterior(const double *theta, int64_t n, const double *t_eval, int32_t t_n,
                             const double *y_obs, const double *span_u0_tol, const double *cov_inv,
                             int64_t max_steps, double *grad_out, int32_t *status, void *stream);
/* Two-phase form of st_lv_grad_log_posterior (same arguments and results, faster): the integration
 * records each accepted step's dense-output polynomial in the workspace and the observation points
 * are evaluated one wave per parameter point; workspace: st_lv_grad_workspace_bytes(n, t_n) bytes
 * of device memory. */
int64_t st_lv_grad_workspace_bytes(int64_t n, int32_t t_n);
int st_lv_grad_log_posterior_ws(const double *theta, int64_t n, const double *t_eval, int32_t t_n,
                                const double *y_obs, const double *span_u0_tol, const double *cov_inv,
                                int64_t max_steps, double *grad_out, int32_t *status, void *workspace,
                                int64_t workspace_bytes, void *stream);
int64_t st_lv_log_density_workspace_bytes(int64_t n, int32_t t_n);
int st_lv_log_target_density(const double *log_theta, const double *theta, int64_t n,
                             const double *t_eval, int32_t t_n, const double *y_obs,
                             const double *span_u0_tol, const double *whiten, double c_log,
                             double norm_logc, int64_t max_steps, double *out, int32_t *status,
                             void *workspace, int64_t workspace_bytes, void *stream);

/* ------------------------------------------------------------------------------------------
 * Integrand protocol -- replaces integrand(ind1, ind2) of the closures returned by
 * stein_thinning.thinning._make_stein_integrand / _make_stein_gf_integrand and
 * stein_thinning.kernel.vfk0_imq (restated at JAX_Stein_Thinning.ipynb cell 27, json ~354-361;
 * Kernel_Stein_discrepancy.ipynb cell 7): out[p] = k(row i1[p], row i2[p]) (weights: w_i1 w_i2).
 * ---------------------------------------------------------------------------------------- */
int st_kernel_pairs(const double *x_soa, const double *g_soa, const double *weights, int64_t ld,
                    int32_t d, double linv_scale, double linv_trace, const int64_t *i1,
                    const int64_t *i2, int64_t n_pairs, double *out, void *stream);

/* ------------------------------------------------------------------------------------------
 * Kernel Stein discrepancy -- replaces stein_thinning.stein.ksd(integrand, n) (called at
 * code/src/utils/ksd.py:27 via calculate_ksd; Gaussian_mixture.ipynb cell 83) and
 * stein_thinning.stein.kmat(integrand, n) (code/tests/test_ksd.py:20; Gaussian_mixture.ipynb
 * cell 94).  Both take a COMPACT problem of m (k) rows (gather the selected rows first).
 * ks_out[i] = sqrt(sum_{a,b <= i} k(a,b)) / (i+1).  kmat_out is the full symmetric (k, k)
 * row-major matrix K[r][c] = k(min(r,c), max(r,c)).
 * ---------------------------------------------------------------------------------------- */
int64_t st_ksd_workspace_bytes(int64_t m, int64_t ld);   /* ld doubles: the column-sum vector */
int st_ksd_cumulative(const double *x_soa, const double *g_soa, const double *weights, int64_t m,
                      int64_t ld, int32_t d, double linv_scale, double linv_trace, double *ks_out,
                      void *workspace, int64_t workspace_bytes, void *stream);
/*
 * Full-sample KSD at scale, row-sharded across GPUs (the n-length column-sum all-reduce):
 *   st_ksd_colsum:  csum_out[i] = sum_{a in [row_begin, row_end), a < i} k(i, a)   (i < n)
 *                   -- the 2*np.sum(k0[:i]) / 2 term of the reference's ksd loop restricted to a
 *                   row range; ranks cover disjoint row ranges and all-reduce (sum) csum;
 *   st_ksd_finish:  ks_out[i] = sqrt(sum_{a <= i} (2 csum[a] + k(a, a))) / (i + 1).
 * st_ksd_cumulative == st_ksd_colsum over [0, m) followed by st_ksd_finish.
 * Summation order differs from the reference's NumPy pairwise sums (floating-point tolerance).
 */
int st_ksd_colsum(const double *x_soa, const double *g_soa, const double *weights, int64_t n,
                  int64_t ld, int32_t d, double linv_scale, double linv_trace, int64_t row_begin,
                  int64_t row_end, double *csum_out, void *stream);
int st_ksd_finish(const double *x_soa, const double *g_soa, const double *weights, int64_t n,
                  int64_t ld, int32_t d, double linv_scale, double linv_trace, const double *csum,
                  double *ks_out, void *stream);

int st_kmat(const double *x_soa, const double *g_soa, const double *weights, int64_t k,
            int64_t ld, int32_t d, double linv_scale, double linv_trace, double *kmat_out,
            void *stream);

/* ------------------------------------------------------------------------------------------
 * Energy distance -- replaces dcor.energy_distance(x, y) (V-statistic, exponent 1) as used by the
 * reference's fit_quality (code/notebooks/lotka_volterra/Comparison.ipynb cell 19,
 * Gradient_free_Student_t.ipynb; Gaussian_mixture.ipynb cells 63-71):
 *   out[i] = sum_{b in [b_begin, b_end), (!triangle or b < i)} ||A_i - B_b||_2,   i < na
 * A, B SoA (d, lda) / (d, ldb); triangle = 1 requires B == A (strict lower triangle: self sums).
 * ED(x, y) = 2 sum(out(x; y)) / (nx ny) - 2 sum(out(x; x, tri)) / nx^2 - 2 sum(out(y; y, tri)) / ny^2.
 * ---------------------------------------------------------------------------------------- */
int st_distance_colsum(const double *a_soa, int64_t lda, int64_t na, const double *b_soa,
                       int64_t ldb, int64_t nb, int32_t d, int64_t b_begin, int64_t b_end,
                       int32_t triangle, double *out, void *stream);
/* The same with the B range split over blockIdx.y chunks (~32768 blocks in all, st_tune key 14: a
 * short A -- e.g. the 1 000 selected points against a 2e5-point validation sample -- still fills
 * the chip, and a long triangle is dealt to the CUs in many small units): the chunk
 * partials go to `workspace` (st_distance_workspace_bytes(na, b_begin, b_end) bytes, 16-B aligned;
 * 0 means no split) and are summed per point in chunk order (deterministic). */
int64_t st_distance_workspace_bytes(int64_t na, int64_t b_begin, int64_t b_end);
int st_distance_colsum_ws(const double *a_soa, int64_t lda, int64_t na, const double *b_soa,
                          int64_t ldb, int64_t nb, int32_t d, int64_t b_begin, int64_t b_end,
                          int32_t triangle, double *out, void *workspace, int64_t workspace_bytes,
                          void *stream);

/* ------------------------------------------------------------------------------------------
 * Host-side input preparation -- stein_thinning.thinning._validate_and_standardize (restated at
 * JAX_Stein_Thinning.ipynb cells 15-18): NaN / inf checks, then per-dimension
 * loc = mean(x, 0), scl = mean(|x - loc|, 0), x / scl, g * scl, bit-identical to the NumPy
 * expressions (their reduction orders reproduced).  Row-major (n, d) host arrays; outputs may
 * alias the inputs.  *status: 0 ok, 1 NaN, 2 inf, 3 a zero scale.  No HIP calls.
 * ---------------------------------------------------------------------------------------- */
int st_standardize_host(const double *sample, const double *gradient, int64_t n, int32_t d,
                        int32_t standardize, double *sample_out, double *gradient_out,
                        double *loc_out, double *scl_out, int32_t *status);

/* scipy.spatial.distance.pdist(rows) (euclidean) of row-major (k, d) device rows into out
 * (k (k - 1) / 2 doubles, scipy's condensed order), bit-identical to scipy 1.15: the 'med'
 * preconditioner's median heuristic (stein_thinning.kernel.make_precon, report.tex:432) sorts them on
 * the device.  2 <= k <= 65535. */
int st_pdist(const double *rows, int64_t k, int32_t d, double *out, void *stream);

/* ------------------------------------------------------------------------------------------
 * Repeated-row compaction (stein_thinning.device.DeviceProblem.dedup_view; no reference
 * counterpart -- an exact shortcut in front of st_greedy).  A row equal bit for bit (x, g, w) to the
 * row before it ties with its run's first row at every step of _greedy_search
 * (JAX_Stein_Thinning.ipynb:281-295) and loses the tie to the lower index, so st_greedy on the run
 * starts, mapped back through rows_out, returns the same indices.
 *   st_run_starts:  starts_out[i] = 1 iff row i starts a run (n bytes); the number of runs lands in
 *                   the first 8 bytes of `workspace` (int64; st_run_workspace_bytes(n), 16-B aligned);
 *   st_run_compact: after the caller read that count: the run starts into (d, ld_out) SoA arrays
 *                   x_out / g_out (and w_out when weights is non-NULL) in row order, rows_out[k] = the
 *                   source row of compact row k (int32), rows [count, ld_out) zeroed.
 * n < 2^31.  Same stream for both calls.
 * ---------------------------------------------------------------------------------------- */
int64_t st_run_workspace_bytes(int64_t n);
int st_run_starts(const double *x_soa, const double *g_soa, const double *weights, int64_t n, int32_t d,
                  int64_t ld, uint8_t *starts_out, void *workspace, int64_t workspace_bytes, void *stream);
int st_run_compact(const double *x_soa, const double *g_soa, const double *weights, int64_t n, int32_t d,
                   int64_t ld, const uint8_t *starts, const void *workspace, int64_t count, int64_t ld_out,
                   double *x_out, double *g_out, double *w_out, int32_t *rows_out, void *stream);

/* The same with the upload underneath: thread 0 computes loc / scl (st_standardize_host's column
 * passes, bit-identical) while the other threads copy the RAW arrays into the page-locked staging
 * buffers stage_x / stage_g (16-B aligned, n d doubles; g's NaN / inf scan fused in) and queue each
 * copied chunk's host-to-device copy into dev_x / dev_g (row-major) on `stream`.  The caller scales
 * on the device (st_layout_soa_scaled with loc_out / scl_out).  d = 2 .. 8 and n >= 65536 only
 * (ST_ERR_UNSUPPORTED otherwise: use st_standardize_host); *status as st_standardize_host's (on a
 * nonzero status the queued copies have finished when it returns). */
int st_standardize_upload(const double *sample, const double *gradient, int64_t n, int32_t d,
                          double *stage_x, double *stage_g, double *dev_x, double *dev_g,
                          double *loc_out, double *scl_out, int32_t *status, void *stream);

/* The device-resident counterpart (the drop-in thin called with ROCm tensors; replaces the reference's
 * np.asarray of the inputs + _validate_and_standardize's statistics): x (row-major (n, d) on the device)
 * comes back into the page-locked stage_x in 64 K-row chunks on `stream`, each chunk's column sums taken
 * as it lands (NumPy's sequential axis-0 order, bit-identical); loc_out / scl_out as st_standardize_host's.
 * g stays on the device (its NaN / inf check is the caller's).  *status: 0 ok, 1 NaN in x, 2 inf in x, 3 a
 * zero scale.  Any n >= 1, d >= 1 (outside d = 2 .. 8, n >= 65536: one copy, then st_standardize_host's
 * column passes; d = 1 assumes NumPy's default bufsize).  Returns when x is on the host and the
 * statistics are done. */
int st_standardize_download(const double *dev_x, int64_t n, int32_t d, double *stage_x, double *loc_out,
                            double *scl_out, int32_t *status, void *stream);

/* row-major (n, d) -> SoA (d, ld) layout helper (device to device) */
int st_layout_soa(const double *rowmajor, int64_t n, int32_t d, int64_t ld, double *soa,
                  void *stream);
/* the same with x / scale[k] (divide = 1) or x * scale[k] (divide = 0) per element: the scaling of
 * _validate_and_standardize on the device (scale: d doubles in device memory) */
int st_layout_soa_scaled(const double *rowmajor, int64_t n, int32_t d, int64_t ld, const double *scale,
                         int32_t divide, double *soa, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* STEIN_THINNING_HIP_H */
