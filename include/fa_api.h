/*
 * fa_api.h — C ABI of the MI355X (gfx950) fused flash-attention op.
 *
 * This is the drop-in boundary.  It replaces the reference's internal C++
 * launcher boundary
 *     cuda_launch::FlashAttentionLauncher<T, RefShape, OrderMap, Policy>::Forward / ::Backward
 *     (/root/reference/flash_attention/kernel/flash_attention.h:220-260,
 *      instantiated at flash_attention.cu:2450-2487)
 * which the TF op kernels call from
 *     FlashAttentionForwardBase::Compute   (flash_attention_forward.cc:280-386)
 *     FlashAttentionBackwardBase::Compute  (flash_attention_backward.cc:181-344)
 * and the FLOP estimator ops
 *     FlashAttentionForwardFlopsEstimationBase::Compute (flash_attention_forward.cc:420-473).
 *
 * Instead of templates over (dtype, seq dims, policy) the ABI takes them as
 * plain enums, and instead of CuTe order-map types it takes the raw sequence
 * shapes plus the sync-mode name: the sync map (sync_methods.cc:8-117) is
 * computed inside the library.  Plain pointers and sizes only; no torch/TF
 * types; no C++ exceptions cross it.
 *
 * Memory layout (channel-first, row-major, exactly the reference's):
 *   Q  [b][d  ][nq]   K [b][d][nk]   V [b][v_d][nk]
 *   O  [b][v_d][nq]   l [b][nq]      m [b][nq]
 * where b = prod(batch shape), nq = prod(Q sequence shape), nk likewise.
 * T is fp16 / fp32 / fp64; l has type L_T = fp32 for fp16 inputs, T otherwise
 * (flash_attention.h:181-185).  All buffers are device memory owned by the
 * caller.  Every output element is written by the library (no caller memset).
 *
 * Threading: every entry point is reentrant; all work is enqueued on `stream`
 * (a hipStream_t, NULL = default stream) with no host synchronisation, so the
 * calls are safe inside hipGraph capture.
 */
#ifndef TF_FLASH_ATTENTION_AMD_FA_API_H_
#define TF_FLASH_ATTENTION_AMD_FA_API_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* dtype of Q/K/V/O/m (and l unless fp16) */
enum fa_dtype { FA_F16 = 0, FA_F32 = 1, FA_F64 = 2 };

/* attention policy = masking rule (flash_attention.h:45-149) */
enum fa_policy { FA_FULL = 0, FA_CAUSAL = 1, FA_LOCAL = 2 };

/* sync mode (sync_methods.cc:113-117) */
enum fa_sync_mode { FA_NONE_FRONT = 0, FA_SCALE_FRONT = 1, FA_SCALE_END = 2 };

/* status codes: 0 = success, >0 = hipError_t passed through, <0 = library errors */
enum fa_status {
  FA_OK = 0,
  FA_ERR_INVALID_ARGUMENT = -1,
  FA_ERR_UNSUPPORTED = -2,
  FA_ERR_WORKSPACE_TOO_SMALL = -3,
};

/* Problem description shared by all entry points.
 * q_seq / k_seq hold `seq_dims` extents in the tensors' axis order
 * (e.g. {H, W} for 2d).  window_size >= 1 and 0 <= log2_stride_size < 31 are
 * only read for FA_LOCAL (attrs of the Local ops, flash_attention_forward.cc:173-175). */
typedef struct fa_problem {
  int32_t dtype;            /* enum fa_dtype */
  int32_t policy;           /* enum fa_policy */
  int32_t seq_dims;         /* 1 or 2 */
  int32_t sync_mode;        /* enum fa_sync_mode */
  int64_t b;                /* flattened batch (batch dims incl. heads) */
  int32_t q_seq[2];
  int32_t k_seq[2];
  int32_t d;                /* Q/K channels */
  int32_t v_d;              /* V/O channels */
  int32_t window_size;
  int32_t log2_stride_size;
  int32_t is_causal;
} fa_problem;

/* "none_front" | "scale_front" | "scale_end" -> enum value, or -1
 * (SyncMethods::Lookup, sync_methods.h:91-101). */
int fa_sync_mode_from_string(const char* name);

/* Validates a problem (ranks, extents, local attrs).  Returns FA_OK or
 * FA_ERR_INVALID_ARGUMENT; the message is available via fa_last_error(). */
int fa_validate(const fa_problem* p);

/* Forward: writes O, l, m.  Replaces FlashAttentionLauncher::Forward
 * (flash_attention.h:225-234) + the 4 memsets of flash_attention_forward.cc:352-369. */
int fa_forward(void* stream, const fa_problem* p,
               const void* Q, const void* K, const void* V,
               void* O, void* l, void* m);

/* Bytes of device scratch fa_backward needs (replaces the Br_occupancy temp,
 * flash_attention_backward.cc:274-283).  Pass that many bytes (or more). */
size_t fa_backward_workspace_bytes(const fa_problem* p);

/* Backward: writes dQ, dK, dV from Q, K, V, O, l, m, dO.  Replaces
 * FlashAttentionLauncher::Backward (flash_attention.h:236-246). */
int fa_backward(void* stream, const fa_problem* p,
                const void* Q, const void* K, const void* V,
                const void* O, const void* l, const void* m, const void* dO,
                void* dQ, void* dK, void* dV,
                void* workspace, size_t workspace_bytes);

/* Algorithmic forward FLOPs 2*(d+v_d)*P, P = rule-allowed (q,k) pairs summed
 * over b (host-only; replaces EstimateForwardFlops, flash_attention.cu:2069-2144,
 * which counted issued tiles instead). */
double fa_estimate_forward_flops(const fa_problem* p);

/* Number of rule-allowed (q,k) pairs for one batch slice (host-only). */
int64_t fa_allowed_pairs(const fa_problem* p);

/* Host-side rule inspection (tests / tooling; no device work).
 * fa_rule_mask: writes nq*nk bytes (1 = pair attended) for one batch slice,
 *   evaluated with the same fa_rules.h code the kernels run.
 * fa_rule_probe: for Q rows [q0,q1] and K cols [k0,k1] (inclusive) writes
 *   out[0..1] = K index range [kb,ke) the kernels visit for that Q block,
 *   out[2..3] = Q index range [qb,qe) visited for that K block,
 *   out[4]    = tile class (0 none allowed, 1 mixed, 2 all allowed). */
int fa_rule_mask(const fa_problem* p, uint8_t* mask);
int fa_rule_probe(const fa_problem* p, int32_t q0, int32_t q1, int32_t k0, int32_t k1, int32_t* out);

/* Human-readable text for a status code / the calling thread's last error. */
const char* fa_error_string(int status);
const char* fa_last_error(void);

/* Library build identifier (kernel variants compiled in). */
const char* fa_build_info(void);

#ifdef __cplusplus
}
#endif

#endif /* TF_FLASH_ATTENTION_AMD_FA_API_H_ */
