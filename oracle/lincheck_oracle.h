/*
 * lincheck_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of the Knossos `:linear` just-in-time linearization search
 * (knossos.linear/analysis, Lowe 2017) as called by this suite's checkers:
 *   - cas-register:  src/jepsen/jgroups/workload/register.clj:106-111 (model (model/cas-register))
 *   - CounterModel:  src/jepsen/jgroups/workload/counter.clj:100-137
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (jepsen-jgroups-raft_amd/csrc) never links or calls this code.
 *
 * Parity pinning: counter model — pinned by the reference's own three known-answer
 * histories (test/jepsen/jgroups/raft_test.clj:6-65, verdict only). cas-register —
 * PARITY UNPINNED against Knossos (no reference test covers it; Knossos is not
 * available in this image); pinned only by hand-derived KATs and a brute-force
 * permutation checker (tests/brute.py).
 */
#ifndef LINCHECK_ORACLE_H
#define LINCHECK_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Shared encoding (same constants as include/lincheck.h; data, not code). */
enum { OR_MODEL_CAS_REGISTER = 1, OR_MODEL_COUNTER = 2, OR_MODEL_LEADER = 3 };
enum { OR_INVOKE = 0, OR_OK = 1, OR_FAIL = 2, OR_INFO = 3 };
enum { OR_F_READ = 0, OR_F_WRITE = 1, OR_F_CAS = 2, OR_F_ADD = 3, OR_F_DECR = 4,
       OR_F_ADD_AND_GET = 5, OR_F_DECR_AND_GET = 6, OR_F_INSPECT = 7 };
enum { OR_V_NIL = 0, OR_V_SCALAR = 1, OR_V_PAIR = 2 };

typedef struct {
  int32_t valid;          /* 1 true, 0 false, 2 unknown */
  int32_t err_code;       /* 0 ok; <0 error (valid == 2) */
  int64_t fail_idx;       /* :index of the :ok completion that could not be linearized, -1 */
  int64_t fail_inv_idx;   /* :index of that op's invocation, -1 */
  int64_t prev_ok_idx;    /* :index of the last :ok completion before fail_idx, -1 */
  int64_t explored;       /* explored_total (SURVEY §8(a) contract) */
  int64_t max_frontier;   /* max |frontier| after any RETURN (and the initial 1) */
  int64_t n_returns;      /* RETURN events processed */
  int64_t final_frontier; /* |frontier| at end (or before the failing RETURN) */
  int64_t n_fail_cfgs;    /* |frontier| just before the failing RETURN */
  int32_t n_pending_at_fail;
  int32_t _pad;
  int64_t wall_ns;        /* oracle_check_many: this history's wall time on its thread */
  int64_t pending_inv_idx[64]; /* invocation :index of each pending op at failure (bit order) */
  char err[128];
} oracle_result;

/* Check one history. Arrays have n entries; index may be NULL (then position is used).
 * On failure, up to cfg_cap pre-failure configs are written as (value, nil, mask, last)
 * where mask bit b refers to pending_inv_idx[b] and last is the :index of the :ok completion
 * of the op the config linearized last (-1: none; Knossos's per-config :last-op [ext]). */
int32_t oracle_check(int32_t model_kind, int64_t init_value, int64_t n,
                     const int64_t* index, const int32_t* process, const int8_t* type,
                     const int8_t* f, const int64_t* v0, const int64_t* v1,
                     const int8_t* vflags, int64_t max_configs, oracle_result* out,
                     int64_t cfg_cap, int64_t* cfg_value, int8_t* cfg_nil,
                     uint64_t* cfg_mask, int64_t* cfg_last);

/* Check n_hist concatenated histories (hist_off has n_hist+1 entries) on n_threads
 * POSIX threads (one history per task). */
int32_t oracle_check_many(int32_t model_kind, int64_t init_value, int32_t n_hist,
                          const int64_t* hist_off, const int64_t* index,
                          const int32_t* process, const int8_t* type, const int8_t* f,
                          const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                          int64_t max_configs, int32_t n_threads, oracle_result* out);

/* Sound counter bounds pre-filter (restates the scan the GPU bounds kernel computes).
 * Returns 1 if every observation is within its [lo, hi] window, 0 if one is not
 * (then *bad_idx = :index of the first offending completion in history order). */
int32_t oracle_counter_bounds(int64_t init_value, int64_t n, const int64_t* index,
                              const int32_t* process, const int8_t* type, const int8_t* f,
                              const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                              int64_t* bad_idx);

int32_t oracle_result_size(void);

#ifdef __cplusplus
}
#endif
#endif
