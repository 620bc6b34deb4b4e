/*
 * lincheck.h — C-ABI of the MI355X linearizability checker (liblincheck.so).
 *
 * Drop-in for the reference's analysis call on its hot path:
 *   (checker/linearizable {:model (model/cas-register) :algorithm :linear})
 *       src/jepsen/jgroups/workload/register.clj:109-111 (inside independent/checker, :106)
 *   (checker/linearizable {:model (CounterModel. 0) :algorithm :linear})
 *       src/jepsen/jgroups/workload/counter.clj:133-137 (model CounterModel, :100-127)
 * Both construct a jepsen.checker/Checker whose (check test history opts) runs
 * knossos.linear/analysis [ext] and returns {:valid? ...}. A JVM caller binds these entry
 * points through JNA; Python binds them through ctypes (lincheck/_lib.py).
 *
 * Conventions: plain C types only; inputs are caller-owned and read-only during the call;
 * outputs are caller-allocated. Every entry point returns 0 on success or a negative
 * LC_E_* code and writes a NUL-terminated message into err (when err_len > 0). Nothing is
 * thrown or aborted across the ABI. The library is thread-safe (one mutex per device).
 *
 * History encoding (one op per entry, all histories concatenated, hist_off[n_hist+1]):
 *   type  : 0 :invoke, 1 :ok, 2 :fail, 3 :info
 *   f     : 0 :read, 1 :write, 2 :cas, 3 :add, 4 :decr, 5 :add-and-get, 6 :decr-and-get,
 *           7 :inspect
 *   vflags: 0 nil, 1 scalar (v0), 2 pair [v0 v1]
 *   LeaderModel (:inspect, leader.clj:63-75): value [leader term] as a pair with v0 = the
 *           caller's id for the leader (-1 for nil and for "null", which serialize-leader makes
 *           equal, leader.clj:51-54; ids equal iff the serialized names are) and v1 = the term;
 *           a nil value is (leader nil, term nil), as destructuring nil gives
 *   index : the op's :index (NULL -> position within its history)
 * Only client ops (integer :process) may be passed; the encoder namespace drops the rest.
 */
#ifndef LINCHECK_H
#define LINCHECK_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LC_ABI_VERSION 6  /* 2: lc_failure_configs gained last_op / out_last_op; 3: LC_MODEL_LEADER;
                            4: LC_H_ABORTED, statistics 34..38 (counter closure tables);
                            5: statistic 42 (counter tile teams), failure configs of histories
                               on the HBM tables (no LC_E_CONFIGS for their width);
                            6: HBM tables to live width 36 in slabs, statistic 43; counters
                               on HBM tables (widths 25..38) */

enum lc_model { LC_MODEL_CAS_REGISTER = 1, LC_MODEL_COUNTER = 2, LC_MODEL_LEADER = 3 };
enum lc_valid { LC_INVALID = 0, LC_VALID = 1, LC_UNKNOWN = 2 };
enum lc_error {
  LC_OK = 0,
  LC_E_ARG = -1,       /* bad argument */
  LC_E_DEVICE = -2,    /* no usable HIP device / HIP runtime error */
  LC_E_MEMORY = -3,    /* device memory exhausted */
  LC_E_INTERNAL = -9,  /* kernel watchdog / internal consistency failure */
  LC_E_CONFIGS = -10,  /* lc_failure_configs: the pre-failure frontier outgrew the dump capacity */
};
/* per-history error codes reported through out_err (valid == LC_UNKNOWN) */
enum lc_hist_error {
  LC_H_OK = 0,
  LC_H_MALFORMED = -4,  /* completion without invocation, double invocation, unknown :type */
  LC_H_WIDE = -5,       /* more concurrently pending ops than the packed key holds */
  LC_H_MODEL = -6,      /* op the model cannot step (unknown :f, wrong value shape, overflow) */
  LC_H_CAPACITY = -7,   /* frontier/closure exceeded max_configs or device capacity */
  LC_H_ABORTED = -8,    /* a device-wide search was stopped by its barrier watchdog (its grid was not
                           wholly resident: another user of the device); undecided, the other
                           histories of the call keep their answers */
};
/* flags */
#define LC_FLAG_BOUNDS_ONLY 0x1 /* counter: run only the bounds pre-filter (sound rejection) */
#define LC_FLAG_NO_BOUNDS 0x2   /* counter: skip the bounds pre-filter */

int32_t lc_abi_version(void);

/* Number of visible HIP devices (0 when none). */
int32_t lc_device_count(void);

/*
 * Check n_hist histories against the model (knossos.linear semantics).
 *   model_kind   : LC_MODEL_CAS_REGISTER (initial value nil; init_value ignored),
 *                  LC_MODEL_COUNTER (initial value init_value) or LC_MODEL_LEADER (the
 *                  :election workload's (LeaderModel. {}), leader.clj:63-85: the empty term ->
 *                  leader map; init_value ignored). A LeaderModel state is the set of
 *                  (term, leader) pairs of the ops linearized so far; a pair can only conflict
 *                  with pairs of its own term, so the search tracks the pairs of terms that
 *                  carry two or more leaders in the history (at most 64 per history, else
 *                  LC_UNKNOWN with LC_H_CAPACITY)
 *   n_gpus       : shards to spread histories over (<=0: one per visible device; more
 *                  shards than devices are multiplexed); results do not depend on it
 *   max_configs  : per-history cap on |frontier| + |closure| (<=0: device capacity only);
 *                  exceeding it reports LC_UNKNOWN with LC_H_CAPACITY (Knossos gives
 *                  :valid? :unknown when it runs out of memory [ext])
 * Per-history outputs (n_hist entries each; any may be NULL):
 *   out_valid       1 true / 0 false / 2 unknown
 *   out_fail_idx    :index of the :ok completion that could not be linearized, else -1
 *   out_fail_inv    :index of that op's invocation, else -1
 *   out_prev_ok     :index of the last :ok completion before it, else -1
 *   out_explored    explored_total (SURVEY §8(a) contract), configs
 *   out_err         LC_H_* code
 */
int32_t lc_check(int32_t model_kind, int64_t init_value, int32_t n_hist,
                 const int64_t* hist_off, const int64_t* index, const int32_t* process,
                 const int8_t* type, const int8_t* f, const int64_t* v0, const int64_t* v1,
                 const int8_t* vflags, int32_t n_gpus, int64_t max_configs, int32_t flags,
                 int8_t* out_valid, int64_t* out_fail_idx, int64_t* out_fail_inv,
                 int64_t* out_prev_ok, int64_t* out_explored, int32_t* out_err,
                 char* err, int32_t err_len);

/*
 * lc_check keeps one plan per device between calls (device buffers sized to the largest check
 * so far, streams, occupancy). lc_release frees the cached plan of `device` (< 0: every
 * device) and its device memory; the next lc_check rebuilds it. A long-lived caller (the JVM)
 * calls it after a large check; it is never done by a static destructor at process exit. It
 * also frees the calling thread's host encoder buffers (kept between that thread's calls).
 * Not part of the reference interface (Knossos keeps no device state).
 */
int32_t lc_release(int32_t device);
/* Statistics (lc_plan_stats layout, below) of the last lc_check shard run on `device`'s cached
 * plan; LC_E_ARG when that device has not run one. */
int32_t lc_check_stats(int32_t device, double* stats, int32_t n);

/*
 * The split lc_check uses for n_gpus > 1 (SURVEY §8(e) axis 1; jepsen.independent's per-key
 * parallelism, register.clj:106): longest-processing-time over n_shards by entry count,
 * out_shard[h] = shard of history h. Host-only (no device needed); deterministic. lc_check
 * runs shard g on device g % (visible devices), so n_gpus may exceed the device count.
 */
int32_t lc_shard_histories(int32_t n_hist, const int64_t* hist_off, int32_t n_shards,
                           int32_t* out_shard);
/*
 * The split lc_check(n_gpus > 1) uses: longest-processing-time over n_shards by each history's
 * modeled time (host encode, then the dense kernels' per-step models summed over the history's
 * RETURN steps: a GPU holding a few hundred keys lasts as long as its slowest chains, and entry
 * counts say nothing about the frontier width that sets a step's cost). out_cost_us (may be
 * NULL) receives the model per history. Counter histories balance by entry count. Host only.
 */
int32_t lc_shard_histories_by_cost(int32_t model_kind, int64_t init_value, int32_t n_hist,
                                   const int64_t* hist_off, const int64_t* index, const int32_t* process,
                                   const int8_t* type, const int8_t* f, const int64_t* v0, const int64_t* v1,
                                   const int8_t* vflags, int32_t n_shards, int32_t* out_shard,
                                   double* out_cost_us, char* err, int32_t err_len);

/*
 * After lc_check reported history `hist` invalid: the frontier just before the failing :ok,
 * the :configs of a Knossos failure report [ext] (compare as a set; at most k are written, in
 * a fixed order). Config i: model value state[i] (register: nil when is_nil[i]; leader: the
 * bitmask of its contested (term, leader) pairs, the caller rebuilds the map); the pending
 * ops it has linearized, as invocation :index values, in linearized[i*64 .. i*64+n_lin[i]) (its
 * Knossos :pending = the pending ops NOT listed there); last_op[i] = :index of the :ok
 * completion of the op it linearized last (Knossos's per-config :last-op), -1 for the initial
 * config. A RETURN's closure stops where the returning op is linearized, so a config it emits
 * has that op last; a config carried through a RETURN keeps its own; a config reached both
 * ways takes the most recent. *out_last_op = the most recent last op over the whole frontier
 * (the report's top-level :last-op). The pending ops themselves (all of them) are written to
 * pending[0..*n_pending). Valid until the next lc_check on this thread. Returns LC_E_CONFIGS
 * when the frontier could not be dumped whole (the verdict stands; only the report is
 * unavailable). Any output pointer may be NULL.
 */
int32_t lc_failure_configs(int32_t hist, int32_t k, int64_t* state, int8_t* is_nil,
                           int64_t* linearized, int32_t* n_lin, int64_t* last_op, int32_t* n_out,
                           int64_t* pending, int32_t* n_pending, int64_t* out_last_op, char* err,
                           int32_t err_len);

/*
 * Counter bounds pre-filter alone: a parallel prefix scan over the
 * history that rejects any observation outside its [lo, hi] window. Sound, not complete:
 * out_ok = 0 implies not linearizable; out_ok = 1 decides nothing.
 * out_bad_idx = :index of the first offending completion in history order, or -1.
 */
int32_t lc_counter_bounds(int64_t init_value, int32_t n_hist, const int64_t* hist_off,
                          const int64_t* index, const int32_t* process, const int8_t* type,
                          const int8_t* f, const int64_t* v0, const int64_t* v1,
                          const int8_t* vflags, int8_t* out_ok, int64_t* out_bad_idx,
                          char* err, int32_t err_len);

/* ---- device-resident counter bounds plans (the C5 bounds scan on HBM-resident inputs) ----
 * One counter history, or one shard of it: the plan owns the observations (reads, *-and-get)
 * completed in entries [own_begin, own_end) and keeps those entries plus the halo back to the
 * earliest owned observation's invocation in HBM. Sharded use (SURVEY §8(e) axis 3): every
 * shard calls lc_bounds_plan_sums (five sums over its owned entries), the shards exchange them
 * (one all-gather of 5 x int64 per shard), and each runs with the sums of all entries before
 * its own_begin. Unsharded: own = [0, n), excl_sums = NULL. out_bad_idx = :index of the first
 * owned completion proven out of bounds (-1 if none); a pass proves nothing (sound rejection).
 * A plan is used by one thread at a time. */
typedef struct lc_bounds_plan lc_bounds_plan;
int32_t lc_bounds_plan_create(int32_t device, int64_t init_value, int64_t n, const int64_t* index,
                              const int32_t* process, const int8_t* type, const int8_t* f,
                              const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                              int64_t own_begin, int64_t own_end, lc_bounds_plan** out, char* err,
                              int32_t err_len);
int32_t lc_bounds_plan_sums(lc_bounds_plan* p, int64_t* out_sums /*[5]*/, char* err, int32_t err_len);
int32_t lc_bounds_plan_run(lc_bounds_plan* p, const int64_t* excl_sums /*[5] or NULL*/, int8_t* out_ok,
                           int64_t* out_bad_idx, double* out_ms, char* err, int32_t err_len);
void lc_bounds_plan_destroy(lc_bounds_plan* p);

/* ---- device-resident plans (benchmarking / repeated runs on HBM-resident inputs) ---- */
typedef struct lc_plan lc_plan;

/* Encode histories on the host and upload them to device `device`. */
int32_t lc_plan_create(int32_t device, int32_t model_kind, int64_t init_value, int32_t n_hist,
                       const int64_t* hist_off, const int64_t* index, const int32_t* process,
                       const int8_t* type, const int8_t* f, const int64_t* v0,
                       const int64_t* v1, const int8_t* vflags, int64_t max_configs,
                       lc_plan** out, char* err, int32_t err_len);
/* Run the search on the resident plan (synchronous). */
int32_t lc_plan_run(lc_plan* p, char* err, int32_t err_len);
/* Copy per-history results of the last run (same meaning as lc_check's outputs). */
int32_t lc_plan_results(lc_plan* p, int8_t* out_valid, int64_t* out_fail_idx,
                        int64_t* out_fail_inv, int64_t* out_prev_ok, int64_t* out_explored,
                        int32_t* out_err);
/*
 * Statistics of the last run, written into stats[0..n) (n <= LC_STATS_N):
 *  0 kernel_ms (HIP events around the search launches)   1 launches
 *  2 steps (RETURN levels, batch lock-step)               3 phases (grid barriers)
 *  4 frontier configs read                                5 candidates routed
 *  6 frontier configs written                             7 closure configs inserted
 *  8 config bytes (C)                                     9 algorithmic bytes
 * 10 workgroups                                          11 spill inserts
 * 12 histories decided by the dense closure-table kernels 13 dense kernels' ms (part of 0)
 * 14 dense big kernel ms (its own stream)               15 dense wave kernel ms (its own stream)
 * 16 dense big kernel algorithmic HBM bytes             17 dense big kernel algorithmic LDS bytes
 * 18 dense wave kernel algorithmic HBM bytes            19 dense wave kernel algorithmic LDS bytes
 * 20..24 lc_plan_create phases, host wall ms: 20 encode (a4/a8), 21 first HIP call +
 *    hipSetDevice, 22 streams/events/occupancy queries, 23 uploads, 24 dense step streams
 * 25..27 dense big kernel: frontier configs in, frontier configs out, configs explored
 * 28..30 the same for the dense wave (+ MID) kernel
 * 31 histories decided on closure tables in HBM (wide.hip: cas-register live width 25..36, counters
 *    25..38; counted in 12 too, counters in 34 too)
 * 32 their kernel's ms (part of 0 and 13)
 * 33 their algorithmic HBM bytes: per step and live word, its X, its pulls and its store (8 B each)
 * 34 counter histories decided on closure tables (ctab.hip; counted in 12 too)  35 their kernel's ms
 * 36..38 the counter tables' frontier configs in, frontier configs out, configs explored
 * 39..41 the closure-table kernels' slowest history: its microseconds from dequeue to end (device
 *    clock), its RETURN steps, its live width (a launch bound by one history's chain of steps
 *    lasts about that long)
 * 42 counter histories decided by tile teams (ctab_team_kernel: one history's table over 2^T
 *    workgroups, live width 17..24; counted in 34)
 * 43 slabs of the HBM tables' last launch (2^split: a slab holds <= 2^32 words, so width 36 has 2;
 *    LC_WIDE_SPLIT asks for up to 8)
 */
#define LC_STATS_N 44
int32_t lc_plan_stats(lc_plan* p, double* stats, int32_t n);
void lc_plan_destroy(lc_plan* p);

/* ---- one history, frontier partitioned over ranks (SURVEY §8(e) axis 2) ----
 * A single huge cas-register history searched by `world` ranks (one process per GPU), each
 * owning the configs whose hash maps to it. Replaces the same knossos.linear/analysis call as
 * lc_check (register.clj:109-111) for ONE history, split across GPUs. The library runs each
 * rank's kernels; the caller runs the collectives (lincheck/partition.py: torch.distributed,
 * RCCL over xGMI). Per RETURN step t = 0, 1, ...:
 *   lc_part_step_begin(t)
 *   loop: lc_part_expand -> send_counts[world]; all-gather the counts (stop when every rank's
 *         are all zero); lc_part_pack into the all-to-all input (contiguous by destination);
 *         all-to-all; lc_part_absorb(received)
 *   lc_part_step_end -> this rank's frontier size; all-reduce SUM: 0 => not linearizable at
 *         step t (lc_part_results gives the :index triple and this rank's explored count;
 *         the explored total is the SUM over ranks).
 * `stream` is a hipStream_t (NULL = the default stream); buffers passed in are device memory
 * of `device`. world <= 16; capacity_log2 (<= 26, 0 = 22) sizes each rank's lists (2^c
 * configs) and hash sets (2^(c+1) words). Exceeding it returns LC_H_CAPACITY (-7).
 * A plan is used by one thread at a time. */
typedef struct lc_part lc_part;
int32_t lc_part_create(int32_t device, int32_t model_kind, int64_t init_value, int64_t n,
                       const int64_t* index, const int32_t* process, const int8_t* type,
                       const int8_t* f, const int64_t* v0, const int64_t* v1, const int8_t* vflags,
                       int32_t rank, int32_t world, int32_t capacity_log2, lc_part** out, char* err,
                       int32_t err_len);
/* info[0] RETURN steps, [1] history error (LC_H_*), [2] mask bits, [3] state bits,
 * [4] invocations, [5] list capacity, [6] kernel ns so far (HIP events), [7] algorithmic
 * HBM bytes so far */
int32_t lc_part_info(lc_part* p, int64_t* info, int32_t n);
int32_t lc_part_step_begin(lc_part* p, int64_t t, void* stream, char* err, int32_t err_len);
int32_t lc_part_expand(lc_part* p, void* stream, int64_t* send_counts /*[world]*/, char* err,
                       int32_t err_len);
int32_t lc_part_pack(lc_part* p, void* stream, void* dst, int64_t dst_cap, char* err,
                     int32_t err_len);
/* recv = NULL absorbs this rank's own staged candidates (world 1 only) */
int32_t lc_part_absorb(lc_part* p, void* stream, const void* recv, int64_t n, char* err,
                       int32_t err_len);
int32_t lc_part_step_end(lc_part* p, void* stream, int64_t* out_count, char* err, int32_t err_len);
/* out4[0] this rank's explored count, [1] :index of step t's :ok completion, [2] of its
 * invocation, [3] of step t-1's completion (-1 at t = 0) */
int32_t lc_part_results(lc_part* p, int64_t t, void* stream, int64_t* out4, char* err,
                        int32_t err_len);
/* World 1, device-resident (no host round trip per level): runs the steps of a fresh plan to
 * the end, to max_steps (< 0: all) or to the first failing step, one cooperative launch per
 * step whose workgroups loop over its BFS levels behind grid barriers, each level absorbing
 * its candidates and expanding the new configs at once. Same verdict, failing step and
 * explored count as the step_begin/expand/absorb/step_end protocol (which world > 1 uses).
 * out4[0] steps run, [1] first failing step (-1: none), [2] BFS levels, [3] explored.
 * lc_part_results reads the failing step's :index triple afterwards. */
int32_t lc_part_run(lc_part* p, void* stream, int64_t max_steps, int64_t* out4, char* err,
                    int32_t err_len);
void lc_part_destroy(lc_part* p);

/* The same search in ONE call for a caller without a collective library (a JVM through JNA):
 * the n_ranks ranks are threads of this process, rank r on device r % (visible devices); per
 * BFS level the counts are exchanged in host memory and each receiver pulls its candidates from
 * every sender's staging segment with peer copies (hipMemcpyPeerAsync over xGMI). Outputs as
 * lc_check's for one history (n_ranks <= 0: one rank per visible device; 1: lc_part_run).
 * Frontier capacity grows with the ranks (capacity_log2 per rank, 0 = 22). */
int32_t lc_part_check(int32_t model_kind, int64_t init_value, int64_t n, const int64_t* index,
                      const int32_t* process, const int8_t* type, const int8_t* f, const int64_t* v0,
                      const int64_t* v1, const int8_t* vflags, int32_t n_ranks, int32_t capacity_log2,
                      int8_t* out_valid, int64_t* out_fail_idx, int64_t* out_fail_inv, int64_t* out_prev_ok,
                      int64_t* out_explored, int32_t* out_err, char* err, int32_t err_len);

#ifdef __cplusplus
}
#endif
#endif
