/*
 * socceraction_amd.h — C ABI of the MI355X (gfx950) valuation-path library
 * (libsocceraction_amd.so).  Plain pointers and sizes only: every array pointer
 * below is a *device* pointer (HBM) unless marked [host]; streams are hipStream_t
 * passed as void*.  All calls are asynchronous on the given stream unless noted.
 *
 * The reference (rtelmore/socceraction) is pure Python/pandas and has no native
 * FFI.  Each entry point below replaces the pandas implementation of one
 * reference function on the hot path; the Python drop-in layer
 * (socceraction_amd/_native.py) binds them with ctypes exactly as INTEGRATION.md
 * shows.  Reference citations are file:line into /root/reference.
 *
 * Conventions
 *  - return 0 on success, a negative SA_E* code on failure; sa_last_error()
 *    returns a thread-local message.  No C++ exception crosses this ABI.
 *  - the caller owns every buffer.  Feature output blocks (one per dtype: bool, f64,
 *    i64; see sa_block) are TILED column-major: rows are grouped in tiles of R rows and
 *    element (row j, column c) of a block with C columns lives at
 *        (j / R) * (C * R) + c * R + (j % R)
 *    i.e. each tile is a [C][R] column-major slab ("record batch").  With
 *    R >= round_up(n, 16) there is one tile and the block is plain column-major with
 *    leading dimension R (pandas' 2-D block layout).  Otherwise R must be a multiple of
 *    SA_BOOL_TILE_QUANTUM (bool block) / SA_NUM_TILE_QUANTUM (f64, i64 blocks).  A block
 *    holds ceil(n / R) * C * R elements; rows n.. of the last tile are scratch.
 *  - input columns are length-n arrays, 16-byte aligned.
 *  - ids are uint8 (SPADL type 0-22, result 0-5, bodypart 0-3, period 1-5; atomic
 *    type 0-32); team ids are int32 codes whose equality equals the equality of
 *    the original team ids (a factorisation); coordinates and times are float64.
 */
#ifndef SOCCERACTION_AMD_H
#define SOCCERACTION_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_ABI_VERSION 3
#define SA_MAX_FRAMES 8 /* max frames n_frames == k of explicit-frame mode (windowed mode: any k) */
#define SA_BOOL_TILE_QUANTUM 1024 /* bool block: rows per tile must be a multiple of this */
#define SA_NUM_TILE_QUANTUM 128   /* f64 / i64 blocks: rows per tile must be a multiple of this */

enum sa_status {
  SA_OK = 0,
  SA_EINVAL = -1,   /* bad argument (maps to ValueError) */
  SA_EHIP = -2,     /* HIP runtime error */
  SA_EDATA = -3,    /* input data error, e.g. non-finite xT coordinates (ValueError) */
  SA_ENOMEM = -4,   /* scratch allocation failed */
};

/* One frame of action columns.  SPADL: c0..c3 = start_x, start_y, end_x, end_y.
 * Atomic-SPADL: c0..c3 = x, y, dx, dy.  result_id is ignored for atomic. */
typedef struct sa_frame {
  const double* c0;
  const double* c1;
  const double* c2;
  const double* c3;
  const double* time_seconds;
  const uint8_t* type_id;
  const uint8_t* result_id;
  const uint8_t* bodypart_id;
  const uint8_t* period_id;
  const int32_t* team;
} sa_frame;

/* A batch of actions split into segments (games).
 *  - n_frames == 1: "windowed" mode, the batched game-state path.  Game-state
 *    window i of action j is row max(j - i, segment start) of frames[0]
 *    (reference vaep/features.py:62-88 gamestates), and if home_team != NULL the
 *    coordinates of every window row are flipped when team[j] != home_team[seg]
 *    (vaep/features.py:91-116 play_left_to_right, keyed on the *current* action).
 *  - n_frames == k > 1: "explicit" mode for the module-level transformers that
 *    receive a user-built list of k frames: window i of row j is row j of
 *    frames[i]; no flip (the frames are already flipped).  n_segments must be 1.
 * Module-level reference functions treat a whole frame as ONE segment. */
typedef struct sa_actions {
  int64_t n;
  int64_t n_segments;
  const int64_t* seg_off;   /* [n_segments + 1], seg_off[0] = 0, seg_off[n_segments] = n */
  const int32_t* home_team; /* [n_segments] team code of the home team, or NULL (no flip) */
  int32_t n_frames;
  int32_t atomic;           /* 0 = SPADL, 1 = Atomic-SPADL */
  sa_frame frames[SA_MAX_FRAMES];
  /* optional (NULL = binary search of seg_off): segment of row b * SA_SEG_BLOCK for every
   * block b < ceil(n / SA_SEG_BLOCK), written once per batch by sa_segment_blocks for THIS
   * seg_off and n (a table of another batch gives wrong segments).  The kernels
   * start every wave's segment cursor from it instead of a ~log2(n_segments)-deep chain of
   * dependent loads. */
  const int32_t* seg_of_block;
} sa_actions;

#define SA_SEG_BLOCK 128

/* seg_of_block[b] = the segment holding row b * SA_SEG_BLOCK, b < ceil(n / SA_SEG_BLOCK), from
 * the segment offsets (seg_off[0] = 0 <= ... <= seg_off[n_segments] = n). Asynchronous. */
int sa_segment_blocks(const int64_t* seg_off, int64_t n_segments, int64_t n, int32_t* seg_of_block,
                      void* stream);

/* Feature transformers (reference vaep/features.py, atomic/vaep/features.py). */
enum sa_xfn {
  SA_XFN_ACTIONTYPE = 0,            /* features.py:151-165        i64 x k   */
  SA_XFN_ACTIONTYPE_ONEHOT,         /* features.py:168-186 (atomic: atomic/vaep/features.py:114-132) bool */
  SA_XFN_RESULT,                    /* features.py:189-203        i64 x k   */
  SA_XFN_RESULT_ONEHOT,             /* features.py:206-224        bool 6k   */
  SA_XFN_ACTIONTYPE_RESULT_ONEHOT,  /* features.py:227-247        bool 138k */
  SA_XFN_BODYPART,                  /* features.py:250-264        i64 x k   */
  SA_XFN_BODYPART_ONEHOT,           /* features.py:267-285        bool 4k   */
  SA_XFN_TIME,                      /* features.py:288-314        i64 k + f64 2k */
  SA_XFN_STARTLOCATION,             /* features.py:317-331        f64 2k    */
  SA_XFN_ENDLOCATION,               /* features.py:334-348        f64 2k    */
  SA_XFN_STARTPOLAR,                /* features.py:355-377        f64 2k    */
  SA_XFN_ENDPOLAR,                  /* features.py:380-402        f64 2k    */
  SA_XFN_MOVEMENT,                  /* features.py:405-424        f64 3k    */
  SA_XFN_TEAM,                      /* features.py:430-452        bool k-1  */
  SA_XFN_TIME_DELTA,                /* features.py:455-473        f64 k-1   */
  SA_XFN_SPACE_DELTA,               /* features.py:476-499        f64 3(k-1) */
  SA_XFN_GOALSCORE,                 /* features.py:505-539 (atomic: atomic/vaep/features.py:229-260) i64 3 */
  SA_XFN_LOCATION,                  /* atomic/vaep/features.py:135-149  f64 2k */
  SA_XFN_POLAR,                     /* atomic/vaep/features.py:152-178  f64 2k */
  SA_XFN_MOVEMENT_POLAR,            /* atomic/vaep/features.py:181-200  f64 2k */
  SA_XFN_DIRECTION,                 /* atomic/vaep/features.py:203-226  f64 2k */
  SA_XFN_COUNT
};

/* Where each requested transformer writes: first column index inside the bool,
 * f64 and i64 output blocks (-1 = not requested / no columns of that dtype). */
typedef struct sa_feature_plan {
  int32_t nb_prev_actions;            /* k: any k >= 1 in windowed mode (n_frames == 1);
                                         explicit mode needs n_frames == k <= SA_MAX_FRAMES */
  int32_t bool_col[SA_XFN_COUNT];
  int32_t f64_col[SA_XFN_COUNT];
  int32_t i64_col[SA_XFN_COUNT];
} sa_feature_plan;

/* One output block: device pointer (16-byte aligned), its column count C and rows per
 * tile R (layout above). */
typedef struct sa_block {
  void* data;
  int32_t n_cols;
  int32_t reserved;
  int64_t tile_rows;
} sa_block;

/* ---- VAEP / Atomic-VAEP ------------------------------------------------------
 * Replaces VAEP.compute_features (vaep/base.py:97-116): gamestates + flip + the
 * transformers of `plan`, for every segment of `a` at once.  A block (or its data) may
 * be NULL when the plan writes no column of that dtype. */
int sa_vaep_features(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                     const sa_block* f64_out, const sa_block* i64_out, void* stream);

/* sa_vaep_features that also writes, in the same pass, the xT cell code (sa_xt_cells) of every
 * action for a fit + rate of these actions on the (xt_l, xt_w) grid -- the VAEP + xT step of
 * one batch (BASELINE cfg2 + cfg4) reads the coordinates from HBM once.  SPADL windowed mode;
 * xt_cells: [n] u32, 16-byte aligned. */
int sa_vaep_features_xt(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                        const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l, int32_t xt_w,
                        uint32_t* xt_cells, void* stream);

/* sa_vaep_features with the bool features written as bitmaps instead of a bool block (the
 * on-device VAEP.rate: the tree kernels read one bit per value, 64 instead of 515 B/action
 * written; windowed mode): bitmap c (plan bool column c, c < n_bool_cols) at bool_bits + c * bits_stride, bit i
 * of byte k = row 8k + i (the Arrow layout of sa_pack_bits), rows >= n clear; bits_stride even
 * and >= 2 * ceil(n / 16) (a multiple of 8 for sa_tree_predict_staged). */
int sa_vaep_features_bits(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bool_bits,
                          int64_t bits_stride, int32_t n_bool_cols, const sa_block* f64_out,
                          const sa_block* i64_out, void* stream);

/* sa_vaep_features_bits with the numeric blocks in float32 (same tiled layout, 4-B elements:
 * f32_out holds the plan's f64 columns rounded to nearest, i32f_out its i64 columns converted):
 * the features of the on-device VAEP.rate for xgboost learners, which compare float32 values
 * (the DMatrix conversion), so half the numeric bytes are written and staged.  k <= 3. */
int sa_vaep_features_bits_f32(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bool_bits,
                              int64_t bits_stride, int32_t n_bool_cols, const sa_block* f32_out,
                              const sa_block* i32f_out, void* stream);

/* VAEP.rate's features for xgboost learners as CONDITION bitmaps: bitmap rows [0, n_bool_cols)
 * = the bool features (as sa_vaep_features_bits), rows n_bool_cols + c = split condition c of
 * the learners (bit set = goes right: xgboost's float32 `x < thr` goes left, NaN follows
 * cond_dl[c]); the numeric columns are evaluated in the numeric pass and never written.
 * Condition c belongs to f64 column j for cond_fstart[j] <= c < cond_fstart[j+1] (j < n_f64_cols)
 * or i64 column j for cond_istart[j] <= c < cond_istart[j+1]; bits 16-byte aligned, bits_stride
 * a multiple of 16 bytes >= 16 * ceil(n / 128).  k <= 3; n_f64_cols and n_i64_cols <= 63 (every
 * k <= 3 plan: at most 47 / 15).  The staged walk then reads every
 * condition from these bitmaps (sa_tree_predict_staged with n_num = 0). */
int sa_vaep_features_conditions(const sa_actions* a, const sa_feature_plan* plan, uint8_t* bits,
                                int64_t bits_stride, int32_t n_bool_cols, int32_t n_f64_cols,
                                int32_t n_i64_cols, const int32_t* cond_fstart,
                                const int32_t* cond_istart, const float* cond_thr,
                                const int32_t* cond_dl, int32_t n_cond, void* stream);

/* goalscore alone (vaep/features.py:505-539; atomic/vaep/features.py:229-260): writes the
 * goalscore_team / _opponent / _diff columns col, col+1, col+2 of the i64 block (one wave per
 * segment).  sa_vaep_features computes the columns inside its numeric pass in windowed mode
 * and launches this scan for explicit frames. */
int sa_vaep_goalscore(const sa_actions* a, const sa_block* i64_out, int32_t col, void* stream);

/* Replaces labels.scores / concedes / goal_from_shot (vaep/labels.py:9-116;
 * atomic/vaep/labels.py:9-107): look-ahead of nr_actions (>=1) clamped at each
 * segment's last row.  Any output may be NULL.  Outputs are bool-byte vectors of length
 * >= ld, 16-byte aligned (ld % 16 == 0, ld >= round_up(n, 16)). */
int sa_vaep_labels(const sa_actions* a, int32_t nr_actions, uint8_t* scores, uint8_t* concedes,
                   uint8_t* goal_from_shot, int64_t ld, void* stream);

/* Replaces formula.value (vaep/formula.py:116-151; atomic/vaep/formula.py:116-141)
 * with float64 probabilities; outputs offensive, defensive, vaep: vectors of length
 * >= round_up(n, 4), 16-byte aligned. */
int sa_vaep_formula_f64(const sa_actions* a, const double* p_scores, const double* p_concedes,
                        double* off, double* def, double* val, void* stream);
/* Same with float32 probabilities (the reference keeps the probability dtype). */
int sa_vaep_formula_f32(const sa_actions* a, const float* p_scores, const float* p_concedes,
                        float* off, float* def, float* val, void* stream);

/* compute_labels + formula.value of the same actions in one launch (the tail of a VAEP
 * step: the ids and team codes are read once): exactly sa_vaep_labels then
 * sa_vaep_formula_f64 / _f32 with the same arguments.  Formula outputs need length
 * >= round_up(n, 16) here. */
int sa_vaep_labels_formula_f64(const sa_actions* a, int32_t nr_actions, uint8_t* scores,
                               uint8_t* concedes, uint8_t* goal_from_shot, int64_t ld,
                               const double* p_scores, const double* p_concedes, double* off,
                               double* def, double* val, void* stream);
int sa_vaep_labels_formula_f32(const sa_actions* a, int32_t nr_actions, uint8_t* scores,
                               uint8_t* concedes, uint8_t* goal_from_shot, int64_t ld,
                               const float* p_scores, const float* p_concedes, float* off,
                               float* def, float* val, void* stream);

/* The batch valuation step in one call -- the notebook loop compute_features +
 * compute_labels + formula.value (vaep/base.py:97-137, vaep/formula.py:116-151) over every
 * segment: exactly sa_vaep_features (sa_vaep_features_xt when xt_cells != NULL) followed by
 * sa_vaep_labels_formula_f64 with the same arguments.  With nb_prev_actions <= 3 and
 * nr_actions <= 11 the labels and the formula are computed inside the numeric feature pass
 * (no launch of their own); otherwise the two launches run.  Windowed mode.  With p_scores,
 * p_concedes, off, def and val all NULL: features + labels only (compute_labels, no formula). */
int sa_vaep_step_f64(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                     const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l, int32_t xt_w,
                     uint32_t* xt_cells, int32_t nr_actions, uint8_t* scores, uint8_t* concedes,
                     uint8_t* goal_from_shot, int64_t ld, const double* p_scores,
                     const double* p_concedes, double* off, double* def, double* val, void* stream);
/* sa_vaep_step_f64's numeric pass in launches of chunk_rows rows (a multiple of 512; 0: one
 * launch), each optionally preceded (prefetch != 0) by a pure-read pass that pulls the chunk's
 * inputs into the Infinity Cache: an A/B probe of the pass's read / write turnaround
 * (bench.py --num-chunks).  The numeric pass only (bool_out without columns of the plan); the
 * same outputs bit for bit. */
int sa_vaep_step_f64_chunked(const sa_actions* a, const sa_feature_plan* plan, const sa_block* bool_out,
                             const sa_block* f64_out, const sa_block* i64_out, int32_t xt_l, int32_t xt_w,
                             uint32_t* xt_cells, int32_t nr_actions, uint8_t* scores, uint8_t* concedes,
                             uint8_t* goal_from_shot, int64_t ld, const double* p_scores,
                             const double* p_concedes, double* off, double* def, double* val,
                             int64_t chunk_rows, int32_t prefetch, void* stream);

/* ---- Expected Threat (xthreat.py) --------------------------------------------
 * Count pass over SPADL actions (frames[0] of `a`; segments ignored):
 * shot[c] += shots (type 11) by start cell, goal[c] += successful shots,
 * move[c] += moves (type pass/dribble/cross, any result) by start cell,
 * trans[s*C+e] += successful moves s->e  (xthreat.py:40-67, 74-98, 144-218).
 * Accumulates into the caller's zeroed buffers (RCCL-reducible), C = l*w.
 * NaN start coordinates are dropped from shot/goal/move counts (`_count`); a
 * non-finite coordinate that the reference would cast to int64 sets a flag in
 * *err_flags (device int32), ONE BYTE per flag so that the ranks' flags add up in the same
 * sum all-reduce as the counts (<= 255 ranks; a flag is set when its byte is non-zero):
 * 0x1 = infinite shot start (scoring_prob, action_prob, fit raise), 0x100 = infinite move
 * start (action_prob, move_transition_matrix, fit raise), 0x10000 = NaN move start or
 * non-finite move end (only move_transition_matrix and fit, which cast every move
 * coordinate, raise; such a move is left out of the transition counts). */
int sa_xt_count(const sa_actions* a, int32_t l, int32_t w, int64_t* shot, int64_t* goal,
                int64_t* move, int32_t* trans, int32_t* err_flags, void* stream);

/* sa_xt_count that also writes, per action, the operand of a later rate() of the SAME actions
 * on the same (l, w) grid without interpolation (fit + rate of one frame, xthreat.py:322-345
 * then :408-465): codes[j] = start cell | end cell << 16 for a successful move, 0xFFFFFFFE for
 * a successful move with a non-finite coordinate, 0xFFFFFFFF otherwise.  codes: [n] u32,
 * 16-byte aligned, or NULL; l * w <= 65535.  flags: SA_XT_COUNT_SHARED when the pass runs
 * concurrently with other kernels (smaller workgroups that co-reside with them). */
#define SA_XT_COUNT_SHARED 1
int sa_xt_count_codes(const sa_actions* a, int32_t l, int32_t w, int64_t* shot, int64_t* goal,
                      int64_t* move, int32_t* trans, int32_t* err_flags, uint32_t* codes,
                      int32_t flags, void* stream);

/* xT cell codes: the binning of a fit + rate of the SAME actions on an (l, w) grid with
 * l * w <= SA_XT_CELLS_MAX_C, computed once per action where the coordinates are read anyway
 * (sa_vaep_features_xt, or sa_xt_cells alone) and consumed by sa_xt_count_cells and
 * sa_xt_rate_cells, which then read 4 B per action instead of the 34 B of coordinates and ids.
 * Code (u32): bits 0-11 start cell, 12-23 end cell (xthreat.py:25-37 binning), 24-25 class
 * (1 = shot, type 11; 2 = move: pass / dribble / cross), 26 result == success, 27 NaN in the
 * start coordinates, 28 start not finite, 29 end not finite.  cells: [n] u32, 16-byte aligned.
 * Grids of l * w <= SA_XT_CELLS16_MAX_C (202: the small-grid count; 16 x 12) take a 16-bit code
 * instead, 2 B per action in the first half of the same buffer: s << 8 | e for a successful move
 * with finite coordinates (s, e: start / end cell); 51712 + 2 s + goal for a shot with a finite
 * start; for a move with a finite start 52224 + s when unsuccessful, 52480 + s / 52736 + s with a
 * non-finite end when unsuccessful / successful; 52992 + {0 shot with a NaN start, 1 shot with an
 * infinite start, 2 / 3 move with a NaN start unsuccessful / successful, 4 / 5 move with an
 * infinite start unsuccessful / successful}; 0xFFFF any other action.  sa_xt_count_cells accumulates exactly what sa_xt_count does on those actions (same
 * counts, same err_flags bits); sa_xt_rate_cells equals sa_xt_rate without interpolation (grid
 * = the (w, l) xT surface). */
#define SA_XT_CELLS_MAX_C 4096
#define SA_XT_CELLS16_MAX_C 202
int sa_xt_cells(const sa_actions* a, int32_t l, int32_t w, uint32_t* cells, void* stream);
int sa_xt_count_cells(const uint32_t* cells, int64_t n, int32_t l, int32_t w, int64_t* shot,
                      int64_t* goal, int64_t* move, int32_t* trans, int32_t* err_flags,
                      int32_t flags, void* stream);
int sa_xt_rate_cells(const uint32_t* cells, int64_t n, int32_t l, int32_t w, const double* grid,
                     double* out, int32_t* err_flags, void* stream);

/* Band-owned count of large grids (203 <= C <= ~12000 cells, e.g. 105 x 68; sa_xt_band_shape
 * says whether a grid takes it): the transition counts without global atomics.  sa_xt_count,
 * sa_xt_count_codes and sa_xt_count_cells use it internally for such grids; a fit over several
 * device batches calls, per batch, sa_xt_count_bucket -- one key per counted action, sorted by
 * start-cell band into buckets[n] (u16: the action's bin in its band's R x P histogram,
 * (start cell - band * R) * P + slot, slot = the end cell of a successful move or C / C+1 / C+2
 * for a shot / scored shot / move without a transition; R = rows per band of sa_xt_band_shape,
 * P = C + 3 rounded up to a multiple of 4) with band_off[NB + 1] (int64, device) -- then ONCE sa_xt_count_from_buckets over every batch's buckets, which adds (or with
 * SA_XT_COUNT_OVERWRITE writes) shot / goal / move and the C x C transition counts exactly as
 * sa_xt_count over all the batches would; err_flags as sa_xt_count, set by the bucket call.
 * `cells` (C <= SA_XT_CELLS_MAX_C) replaces the coordinates of `a` when not NULL (then `a` may
 * be NULL and n is the action count); `codes` as in sa_xt_count_codes (coordinates only).
 * buckets / band_off are plain device arrays the caller keeps until the count call.
 * Replaces xthreat.py:40-67 (`_count`) and :177-218 (`move_transition_matrix` counts). */
#define SA_XT_COUNT_OVERWRITE 2
int sa_xt_band_shape(int32_t l, int32_t w, int32_t* rows_per_band, int32_t* n_bands);
int sa_xt_count_bucket(const sa_actions* a, const uint32_t* cells, int64_t n, int32_t l, int32_t w,
                       uint16_t* buckets, int64_t* band_off, int32_t* err_flags, uint32_t* codes,
                       uint64_t* interp_codes, int32_t L, int32_t W, void* stream);
/* The band-owned count of bands [band0, band0 + nbands) only (a rank's row block in the
 * row-sharded multi-GPU fit: its bands' keys gathered from every rank by an all-to-all).  Set k's
 * keys of local band lb (band band0 + lb) are buckets[k][band_off[k][lb] .. band_off[k][lb + 1]),
 * band_off[k] holding nbands + 1 entries; the outputs hold the rows from band0 * R on (R from
 * sa_xt_band_shape): shot / goal / move_rows [min(nbands R, C - band0 R)], trans_rows
 * [that many rows x C].  flags: SA_XT_COUNT_OVERWRITE or 0 (add). */
int sa_xt_count_band_rows(int32_t nsets, const uint16_t* const* buckets,
                          const int64_t* const* band_off, int32_t l, int32_t w, int32_t band0,
                          int32_t nbands, int64_t* shot_rows, int64_t* goal_rows,
                          int64_t* move_rows, int32_t* trans_rows, int32_t flags, void* stream);
/* interp_codes (coordinates only; [n] u64, 16-byte aligned, or NULL): per action the operand of a
 * later rate(use_interpolation=True) of the SAME actions on the L x W node grid -- start node |
 * end node << 32 of a successful move, 2^64 - 2 for one with a non-finite coordinate, 2^64 - 1
 * otherwise -- consumed by sa_xt_rate_interp_codes, which then equals sa_xt_rate_interp on those
 * actions bit for bit (values, NaN pattern, err_flags bit 4) reading 8 B per action. */
int sa_xt_rate_interp_codes(const uint64_t* interp_codes, int64_t n, const double* xT,
                            const double* cx, const double* cy, int32_t l, int32_t w,
                            const double* xs, int32_t L, const double* ys, int32_t W, double* out,
                            int32_t* err_flags, void* stream);
/* sa_xt_rate_interp_codes of nsets action sets (a fit's device batches) in one launch per 16
 * sets, the surface staged once: set q's interp_codes[q] / n[q] / out[q] as above, one err_flags
 * for all.  (ExpectedThreat.rate(use_interpolation=True) xthreat.py:443-464 of a fit's
 * batches.) */
int sa_xt_rate_interp_codes_many(int32_t nsets, const uint64_t* const* interp_codes,
                                 const int64_t* n, const double* xT, const double* cx,
                                 const double* cy, int32_t l, int32_t w, const double* xs,
                                 int32_t L, const double* ys, int32_t W, double* const* out,
                                 int32_t* err_flags, void* stream);
/* ExpectedThreat.fit + rate(use_interpolation=True) of the same actions (xthreat.py:322-345,
 * 408-465) in one call, for grids above the small-grid limit: sa_xt_solve_ex (no transposed
 * matrix; ell / row_len the count's compact rows or NULL) then sa_xt_rate_interp_codes_many over
 * the surface mats[3 * C ..] -- the rate queued right behind the one-launch reordered solve,
 * before the host waits for the solve's status, and run again when the status sends the solve to
 * the reference's order.  The same outputs as the two calls. */
int sa_xt_fit_rate_interp_codes(const int64_t* shot, const int64_t* goal, const int64_t* move,
                                const int32_t* trans, int32_t l, int32_t w, double eps,
                                int32_t max_iter, int32_t flags, double* mats, double* heatmaps,
                                int32_t* n_iter, int32_t* path, const uint32_t* ell,
                                const int32_t* row_len, int32_t nsets,
                                const uint64_t* const* interp_codes, const int64_t* n,
                                const double* cx, const double* cy, const double* xs, int32_t L,
                                const double* ys, int32_t W, double* const* out,
                                int32_t* err_flags, void* stream);
int sa_xt_count_from_buckets(int32_t nsets, const uint16_t* const* buckets,
                             const int64_t* const* band_off, int32_t l, int32_t w, int64_t* shot,
                             int64_t* goal, int64_t* move, int32_t* trans, int32_t flags,
                             void* stream);
/* sa_xt_count_from_buckets that also writes the count rows in the compact form of
 * sa_xt_compact_rows (ell [C * sa_xt_compact_bytes(C, 1) / 4] u32, 16-byte aligned; row_len [C]),
 * straight from the bins: the large-grid solve (sa_xt_solve_ex with ell / row_len) then skips
 * its own build pass over the dense table.  Needs SA_XT_COUNT_OVERWRITE, at most 24 bucket sets
 * and 1025 <= C <= 9472; ell = row_len = NULL is sa_xt_count_from_buckets.
 * flags | SA_XT_COUNT_COMPACT_ONLY (with ell): the dense C x C rows of `trans` are written only
 * for the bands (sa_xt_band_shape's rows per band) that hold a transition count >= 65535 -- the
 * only dense entries the compact solve reads; the other rows are left as they were.  shot / goal
 * / move, ell and row_len are written in full.  (A fit that reads only the compact rows: no
 * 4 C^2-byte flush, 204 MB at 105 x 68.) */
#define SA_XT_COUNT_COMPACT_ONLY 4
int sa_xt_count_from_buckets_ex(int32_t nsets, const uint16_t* const* buckets,
                                const int64_t* const* band_off, int32_t l, int32_t w,
                                int64_t* shot, int64_t* goal, int64_t* move, int32_t* trans,
                                int32_t flags, uint32_t* ell, int32_t* row_len, void* stream);

/* Grids up to SA_XT_SOLVE_MAX_C cells solve in one workgroup from the transposed matrix. */
#define SA_XT_SOLVE_MAX_C 1024

/* Normalise the counts into the reference's matrices and run the value iteration
 * x <- s*p_shot + p_move * (T x) until no cell changes by more than eps
 * (xthreat.py:278-345).  Writes (all float64, device):
 *   mats[4*C] = scoring_prob | shot_prob | move_prob | xT  (row-major w x l each)
 *   trans_t[C*C] = transition matrix TRANSPOSED (trans_t[e*C+s] = T[s,e]); may be NULL when
 *                  C > SA_XT_SOLVE_MAX_C (the large-grid iteration reads the counts directly)
 *   heatmaps[(max_iter+1)*C] = x after 0..n_iter iterations
 * *n_iter [host] receives the iteration count (-1: max_iter reached first).
 * Synchronises the stream. */
int sa_xt_solve(const int64_t* shot, const int64_t* goal, const int64_t* move,
                const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                double* mats, double* trans_t, double* heatmaps, int32_t* n_iter, void* stream);
/* sa_xt_solve (ExpectedThreat.fit xthreat.py:322-345 + __solve :278-320) with a choice of
 * summation order for grids above SA_XT_SOLVE_MAX_C cells (smaller
 * grids always sum in the reference's order, bit-exact).  Large grids by default solve in ONE
 * launch with each row's sum reordered into a fixed parallel tree (run-to-run reproducible)
 * under a rigorous error bound: every `diff > eps` decision, and so the iteration count, is the
 * reference's, and the iterates are within 4e-11 relative of the reference's (26 iterations at
 * 105 x 68); when some cell's diff falls inside the bound the system is re-solved in the
 * reference's order.  flags: SA_XT_SOLVE_EXACT = always the reference's order (bit-exact
 * iterates, one launch per iteration).  *path (may be NULL) receives which path produced the
 * result (SA_XT_PATH_*).  ell / row_len (both or NULL; grids of 1025 - 9472 cells): the compact
 * form of `trans` as sa_xt_count_from_buckets_ex or sa_xt_compact_rows wrote it, used instead of
 * building it again.  Same outputs and synchronisation as sa_xt_solve. */
#define SA_XT_SOLVE_EXACT 1
#define SA_XT_PATH_SEQUENTIAL 0   /* the reference's order (small grid, or SA_XT_SOLVE_EXACT) */
#define SA_XT_PATH_REORDERED 1    /* reordered sums, every decision outside the error bound */
#define SA_XT_PATH_INSIDE_BOUND 2 /* reordered, a decision inside the bound: re-solved in order */
#define SA_XT_PATH_UNAVAILABLE 3  /* reordered solve not launchable here: solved in order */
#define SA_XT_PATH_TIMEOUT 4      /* the reordered solve's grid barrier timed out (another grid held
                                     CUs: 50 ms at the first barrier, 1 s later): solved in order */
int sa_xt_solve_ex(const int64_t* shot, const int64_t* goal, const int64_t* move,
                   const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                   int32_t flags, double* mats, double* trans_t, double* heatmaps, int32_t* n_iter,
                   int32_t* path, const uint32_t* ell, const int32_t* row_len, void* stream);
/* sa_xt_solve for grids of <= SA_XT_SOLVE_MAX_C cells without the host round trip: the
 * iteration count (-1: max_iter reached first) is written to device memory *n_iter_dev and
 * nothing is synchronised, so a consumer of the surface (sa_xt_rate_cells) can be enqueued
 * right behind it (the bench step's side stream). */
int sa_xt_solve_async(const int64_t* shot, const int64_t* goal, const int64_t* move,
                      const int32_t* trans, int32_t l, int32_t w, double eps, int32_t max_iter,
                      double* mats, double* trans_t, double* heatmaps, int32_t* n_iter_dev,
                      void* stream);

/* Normalisation only (scoring_prob, action_prob, move_transition_matrix of
 * xthreat.py:74-218): mats[3*C] = scoring_prob | shot_prob | move_prob, trans_t as in
 * sa_xt_solve.  Asynchronous. */
int sa_xt_normalize(const int64_t* shot, const int64_t* goal, const int64_t* move,
                    const int32_t* trans, int32_t l, int32_t w, double* mats, double* trans_t,
                    void* stream);

/* Row-sharded value iteration (multi-GPU fit of large grids, e.g. 105 x 68: every rank holds
 * the count rows of its own row range after a reduce-scatter and the full x after each
 * all-gather).  sa_xt_probabilities: mats[3*C] = scoring | shot | move probability (as
 * sa_xt_normalize) and gs = scoring * shot, pmove = move probability (xthreat.py:296-297).
 * sa_xt_iterate_rows: one iteration of rows [r0, r0 + nrows): cnt_rows holds their count
 * rows (row r0 + i at cnt_rows + i*C), x the full current vector (length C);
 * x_next_rows[i] = gs + pmove * sum_c (cnt / move[r]) * x[c] in the reference's summation
 * order (xthreat.py:306-317), *flag_out |= some row moved by more than eps; a non-NULL
 * *flag_prev == 0 makes the call a no-op.  Asynchronous. */
int sa_xt_probabilities(const int64_t* shot, const int64_t* goal, const int64_t* move, int32_t C,
                        double* mats, double* gs, double* pmove, void* stream);
int sa_xt_iterate_rows(const int32_t* cnt_rows, const int64_t* move, const double* gs,
                       const double* pmove, int32_t C, int32_t r0, int32_t nrows, const double* x,
                       double eps, double* x_next_rows, const int32_t* flag_prev, int32_t* flag_out,
                       void* stream);
/* The same iteration over a compact form of the count rows built once (C <= 9472; sa_xt_solve
 * uses it for C > SA_XT_SOLVE_MAX_C): sa_xt_compact_rows writes each row's non-zero counts in
 * column order (4 B each: column | min(count, 65535) << 16) in row i's pe = C rounded up to a
 * multiple of 128 slots, the k-th at slot (k & ~127) | (k % 32) << 2 | (k / 32) % 4 (u32,
 * sa_xt_compact_bytes(C, nrows) bytes), and their number at row_len[i] (int32 [nrows], device);
 * sa_xt_iterate_compact then equals sa_xt_iterate_rows bit for bit (cnt_rows: the same dense
 * rows, read only for counts >= 65535).  Asynchronous. */
int64_t sa_xt_compact_bytes(int32_t C, int32_t nrows);
int sa_xt_compact_rows(const int32_t* cnt_rows, int32_t C, int32_t nrows, uint32_t* ell,
                       int32_t* row_len, void* stream);
int sa_xt_iterate_compact(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows,
                          const int64_t* move, const double* gs, const double* pmove, int32_t C,
                          int32_t r0, int32_t nrows, const double* x, double eps,
                          double* x_next_rows, const int32_t* flag_prev, int32_t* flag_out,
                          void* stream);
/* The whole value iteration (__solve xthreat.py:278-320) of a grid from the compact form of ALL
 * its C rows (as built by
 * sa_xt_compact_rows; the multi-GPU fit gathers it from the ranks): heatmaps[(max_iter+1)*C]
 * = x after 0..n_iter iterations, *n_iter [host] the count (-1: max_iter reached first), the
 * summation order chosen by `flags` exactly as in sa_xt_solve_ex (*path may be NULL).
 * cnt_rows: the dense count rows, read only for counts >= 65535.  Synchronises the stream. */
int sa_xt_solve_compact(const uint32_t* ell, const int32_t* row_len, const int32_t* cnt_rows,
                        const int64_t* move, const double* gs, const double* pmove, int32_t C,
                        double eps, int32_t max_iter, int32_t flags, double* heatmaps,
                        int32_t* n_iter, int32_t* path, void* stream);

/* interp2d(x=cx, y=cy, z=xT, kind='linear')(xs, ys) of ExpectedThreat.interpolator
 * (xthreat.py:347-378): grid[r*L + h] = bilinear(xT; xs[h], ys[r]) through the cell
 * centres cx[l], cy[w], clamped to the centre hull (FITPACK evaluation clamps).  All
 * arrays are device f64; xs (length L) and ys (length W) sorted ascending. */
int sa_xt_interp_grid(const double* xT, const double* cx, const double* cy, int32_t l, int32_t w,
                      const double* xs, int32_t L, const double* ys, int32_t W, double* grid,
                      void* stream);

/* ExpectedThreat.rate(use_interpolation=True) (xthreat.py:443-464) WITHOUT materialising the
 * L x W surface: a successful move's start and end node values are evaluated per action from
 * the (w x l) xT surface -- each node's bracket (i, tx) / (j, ty) tabulated once per call by the
 * device function sa_xt_interp_grid uses, then its bilinear expression in the same order -- so
 * out[] equals sa_xt_interp_grid(xT, cx, cy, l, w, xs, L, ys, W) + sa_xt_rate(..., L, W) bit for
 * bit, NaN pattern and err_flags bit 4 included.  Reads 34 B and writes 8 B per action; the
 * surface (w*l doubles) and the (L + W) node tables stay cache-resident.  Replaces the grid
 * gather of `grid[w - 1 - yj, xi]` (xthreat.py:456-464). */
int sa_xt_rate_interp(const sa_actions* a, const double* xT, const double* cx, const double* cy,
                      int32_t l, int32_t w, const double* xs, int32_t L, const double* ys, int32_t W,
                      double* out, int32_t* err_flags, void* stream);

/* ExpectedThreat.rate (xthreat.py:408-465): out[j] = grid[W-1-yj(end), xi(end)] -
 * grid[W-1-yj(start), xi(start)] for successful moves, NaN otherwise.  A non-finite
 * coordinate of a successful move (the reference's int64 cast raises) sets bit 4 in
 * *err_flags (device int32, may be NULL). */
int sa_xt_rate(const sa_actions* a, const double* grid, int32_t L, int32_t W, double* out,
               int32_t* err_flags, void* stream);

/* sa_xt_rate from the codes of sa_xt_count_codes (grid = the fitted (w, l) xT surface):
 * same values and err_flags bit 4 as sa_xt_rate on those actions, reading 4 B per action
 * instead of the coordinates and ids.  out: [n] f64, 16-byte aligned. */
int sa_xt_rate_codes(const uint32_t* codes, int64_t n, const double* grid, double* out,
                     int32_t* err_flags, void* stream);

/* ---- SPADL -> Atomic-SPADL (atomic/spadl/base.py:15-235) ------------------------
 * Replaces convert_to_atomic: the four insertion passes (_extra_from_passes :38-112,
 * spadl/base.py _add_dribbles :54-93, _extra_from_shots :115-165, _extra_from_fouls
 * :168-196), each followed in the reference by a stable sort on (game_id, period_id,
 * action_id), then _convert_columns (:199-220) and _simplify (:223-235).  Every inserted row
 * lands right after the row that produced it, so the whole conversion is one expansion of
 * each input row r (in sorted order) into 1..5 output rows that depends only on r, its
 * input-order successor (first pass) and its sorted-order successor (later passes).
 *
 * Input: SPADL actions as device columns of length n.  game / team / player / event are
 * int32 equality codes of game_id / team_id / player_id / original_event_id (the caller
 * factorises them and decodes the output codes; event -1 = missing).  `order` lists the rows
 * in (game_id, period_id, action_id) order (a stable sort; the keys must be unique), or is
 * NULL when the rows are already in that order. */
typedef struct sa_spadl_frame {
  int64_t n;
  const double* time_seconds;
  const double* start_x;
  const double* start_y;
  const double* end_x;
  const double* end_y;
  const int32_t* game;
  const int32_t* team;
  const int32_t* player;
  const int32_t* event;
  const uint8_t* period_id;   /* 1..5 */
  const uint8_t* type_id;     /* SPADL 0..22 */
  const uint8_t* result_id;   /* 0..5 */
  const uint8_t* bodypart_id; /* 0..3 */
  const int64_t* order;       /* [n] or NULL */
} sa_spadl_frame;

/* Atomic-SPADL output columns (device, length n_out); action_id is the row position. */
typedef struct sa_atomic_frame {
  double* time_seconds;
  double* x;
  double* y;
  double* dx;
  double* dy;
  int32_t* game;
  int32_t* team;
  int32_t* player;
  int32_t* event;             /* -1 = missing (the dribbles of _add_dribbles) */
  uint8_t* period_id;
  uint8_t* type_id;           /* Atomic-SPADL 0..32 */
  uint8_t* bodypart_id;
} sa_atomic_frame;

/* Device scratch the two calls below share (bytes, 16-byte aligned). */
int64_t sa_atomic_scratch_bytes(int64_t n);
/* Pass 1: the output row count of every 1024-row block and their exclusive prefix;
 * *n_out [host] receives the total.  Synchronises the stream. */
int sa_atomic_count(const sa_spadl_frame* in, void* scratch, int64_t* n_out, void* stream);
/* Pass 2: writes the n_out output rows (scratch from sa_atomic_count, same input). */
int sa_atomic_emit(const sa_spadl_frame* in, const void* scratch, const sa_atomic_frame* out,
                   void* stream);

/* ---- _add_dribbles (spadl/base.py:54-93) ------------------------------------------
 * SPADL rows out (device, length n_out): the input columns' codes plus `src`, the input row a
 * row came from (>= 0), or ~q for a dribble inserted before input row q (the successor whose
 * game / team / player / timestamp it carries). action_id is the row position. */
typedef struct sa_spadl_out {
  double* time_seconds;
  double* start_x;
  double* start_y;
  double* end_x;
  double* end_y;
  int32_t* game;
  int32_t* team;
  int32_t* player;
  int32_t* event;             /* -1 = missing (the dribbles) */
  uint8_t* period_id;
  uint8_t* type_id;
  uint8_t* result_id;
  uint8_t* bodypart_id;
  int64_t* src;
} sa_spadl_out;

/* Pass 1 (replaces the shift / predicate half of spadl/base.py:54-69): marks row j (flags[j],
 * optional) when a dribble is inserted between it and its input-order successor, and leaves
 * the per-block output counts and their prefix in scratch (sa_atomic_scratch_bytes(n) bytes);
 * *n_out [host] = n + dribbles. Thresholds: min_dribble_length**2, max_dribble_length**2,
 * max_dribble_duration (spadl/base.py:49-51). in->order must be NULL. With action_id (device,
 * f64 [n], the sort key the reference compares after its concat), *n_misplaced [host,
 * optional] counts the rows that rule out the fast layout of sa_dribble_emit (keys not
 * strictly increasing, or a dribble not sorting between its row and the next); -1 without
 * action_id. Game codes must preserve the game_id order. Synchronises. */
int sa_dribble_count(const sa_spadl_frame* in, double min_len2, double max_len2, double max_dt,
                     const double* action_id, void* scratch, uint8_t* flags, int64_t* n_out,
                     int64_t* n_misplaced, void* stream);
/* Pass 2 (spadl/base.py:71-93): writes the n_out rows in the reference's sorted order.
 * dest == NULL: input keys strictly increasing and every dribble sorting directly after its
 * row (row j at j + dribbles before j, its dribble next); else dest[n_out] is the output
 * position of each concatenated row (the n inputs, then the dribbles in input order). */
int sa_dribble_emit(const sa_spadl_frame* in, double min_len2, double max_len2, double max_dt,
                    const void* scratch, const int64_t* dest, const sa_spadl_out* out, void* stream);

/* ---- convert_to_atomic, general form ----------------------------------------------
 * For frames whose (game_id, period_id, action_id) keys repeat or lie no more than 0.1 apart inside a game and period (then the rows _extra_from_passes inserts do not all
 * sort directly after their parents; base.py:82,109-110).  The first pass runs on its own:
 *   sa_atomic_passes_flags: flags[j] (device u8 [n]) = 1 when input row j gets a receival /
 *     interception / out / offside row (its INPUT-order successor decides, base.py:39-73);
 *     in->order must be NULL.
 *   sa_atomic_passes_emit: writes the n + m rows of the reference's concat (the n inputs, then
 *     the m inserted rows of `parents` [device, the flagged rows in input order]) as SPADL rows
 *     at dest[k] (device int64 [n + m]: the position of concatenated row k in the stable sort
 *     of (game, period, action_id / action_id + 0.1), from the host).  Inserted rows carry
 *     start = end = the parent's end, the midpoint time, bodypart foot, result 255 (the
 *     reference's -1) and the atomic type id; src = input row, or ~parent for an inserted row.
 *   sa_atomic_count_after_passes / sa_atomic_emit_after_passes: sa_atomic_count / emit of that
 *     sorted output (order NULL) without the first pass -- the reference's remaining passes
 *     (_add_dribbles, _extra_from_shots, _extra_from_fouls) and the column conversion. */
int sa_atomic_passes_flags(const sa_spadl_frame* in, uint8_t* flags, void* stream);
int sa_atomic_passes_emit(const sa_spadl_frame* in, const int64_t* parents, int64_t m,
                          const int64_t* dest, const sa_spadl_out* out, void* stream);
int sa_atomic_count_after_passes(const sa_spadl_frame* in, void* scratch, int64_t* n_out,
                                 void* stream);
int sa_atomic_emit_after_passes(const sa_spadl_frame* in, const void* scratch,
                                const sa_atomic_frame* out, void* stream);

/* Segment (game) offsets of a row-sorted key column whose values are exactly 0..n_segments-1,
 * each present -- e.g. the game codes of sa_atomic_emit's output:
 * seg_off[g] = first row of g, seg_off[n_segments] = n. */
int sa_segment_offsets(const int32_t* key, int64_t n, int64_t n_segments, int64_t* seg_off,
                       void* stream);

/* ---- Arrow / Parquet export --------------------------------------------------------
 * The per-game feature and label stores of the notebooks (2-compute-features-and-labels.ipynb:
 * `X.to_hdf(features_h5, f"game_{game_id}")`): bool columns leave the device as Arrow bitmaps
 * (LSB first, rows >= n zero). bits: [n_cols][col_stride] bytes, col_stride even and
 * >= 2*ceil(n/16); the block's tile_rows a multiple of 16 and its data 16-byte aligned. */
int sa_pack_bits(const sa_block* bool_blk, int64_t n, uint8_t* bits, int64_t col_stride, void* stream);

/* ---- gradient-boosted trees on the feature blocks --------------------------------
 * The learner call of VAEP.rate (`_estimate_probabilities`, vaep/base.py:284-294): P(class 1)
 * of a binary gradient-boosted tree ensemble for every row of the feature blocks.
 * nodes: n_nodes records of 24 bytes { double threshold_or_leaf_value; int32 feature (-1 =
 * leaf); int32 left; int32 right | (default_left << 31); int32 pad } with absolute child
 * indices; roots[n_trees] the root node of each tree, summed in that order onto base_margin.
 * feature_slots[f] = (kind << 24) | column locates model feature f in the blocks (kind 0 =
 * bool block, 1 = f64, 2 = i64).  le = 1: `x <= threshold` goes left (scikit-learn), 0:
 * `x < threshold` (xgboost); NaN follows default_left.  f32 = 1: xgboost float32 arithmetic
 * and float output p_out[n], else float64 (scikit-learn).  p = 1 / (1 + exp(-margin)).
 * tree_depth (optional, device, [n_trees]): split levels on each tree's longest root-to-leaf
 * path; with it (and a model that fits LDS) trees are walked a fixed number of levels. */
int sa_tree_predict(const void* nodes, int32_t n_nodes, const int32_t* roots, const int32_t* tree_depth,
                    int32_t n_trees, const int32_t* feature_slots, int32_t n_features,
                    const sa_block* bool_blk, const sa_block* f64_blk, const sa_block* i64_blk, int64_t n,
                    double base_margin, int32_t le, int32_t f32, void* p_out, void* stream);

/* sa_tree_predict with every split turned into a condition bit staged in LDS per workgroup of
 * 512 rows, then a branch-free fixed-depth walk (the same probabilities as sa_tree_predict bit
 * for bit).  Conditions: 0 = never set (constant splits); 1 .. n_bool = bool block column
 * bool_cols[i - 1] is set; 1 + n_bool + c = numeric condition c: the value of the numeric
 * column q with col_start[q] <= c < col_start[q + 1] (num_cols[q] = (kind << 24) | column, kind
 * 1 = f64 block, 2 = i64 block; n_ncol distinct columns, col_start[0] = 0, col_start[n_ncol] =
 * n_num) goes right of num_thr[c] (T; `x <= thr` goes left for le = 1, `x < thr` for le = 0;
 * NaN goes left iff num_dl[c]); 1 + n_bool + n_num <= 65536.  model: nodes, n_nodes (< 65536)
 * uint32 { condition | first child << 16 }: a split's children are adjacent and a row takes
 * first child + its condition bit; leaves are self-loops (condition 0, first child = the leaf);
 * leaf: T[n_nodes] leaf values; roots[n_trees]: each tree's root; tree_depth[n_trees]: split
 * levels of each tree; p_out[n]: the probabilities.  T = float for f32 = 1 (xgboost), else
 * double.  The bool columns come from bool_blk, or -- when bool_bits is not NULL -- from the
 * bitmaps of sa_vaep_features_bits (bool_cols index its bitmaps; bits_stride a multiple of 8).
 * f32 bit 1 (f32 = 3): the f64 / i64 blocks hold float32 values (sa_vaep_features_bits_f32);
 * xgboost arithmetic only (bit 0 set), and the same probabilities bit for bit.
 * sa_tree_staged_lds_bytes: the LDS a model needs at most (<= 160 KiB; n_cond = 1 + n_bool +
 * n_num; the walk also stages the roots and depths, bounded here by n_nodes trees). */
typedef struct sa_tree_model {
  const void* nodes;
  const void* leaf;
  const int32_t* roots;
  const int32_t* tree_depth;
  int32_t n_nodes;
  int32_t n_trees;
  double base_margin;
  void* p_out;
} sa_tree_model;
int64_t sa_tree_staged_lds_bytes(int32_t n_nodes, int32_t n_cond, int32_t f32);
int sa_tree_predict_staged(const sa_tree_model* model, const int32_t* bool_cols, int32_t n_bool,
                           const int32_t* num_cols, const int32_t* col_start, int32_t n_ncol,
                           const void* num_thr, const int32_t* num_dl, int32_t n_num,
                           const sa_block* bool_blk, const uint8_t* bool_bits, int64_t bits_stride,
                           const sa_block* f64_blk, const sa_block* i64_blk, int64_t n, int32_t le,
                           int32_t f32, void* stream);

/* ---- runtime ------------------------------------------------------------------ */
int sa_abi_version(void);
const char* sa_last_error(void);
/* Hash of the sources, headers, compile flags and defines the library was built from
 * (socceraction_amd/build.py); the Python loader refuses a library built from other sources. */
const char* sa_build_id(void);
/* Scratch: sa_xt_solve / sa_xt_normalize take their device scratch from a per-device arena
 * owned by the library (mutex-guarded, reused in stream order); sa_shutdown() waits for the
 * last use of every slot and frees the arena.  The library stays usable afterwards. */
int sa_shutdown(void);
/* Device memory for output blocks: flags bit 0 = physically contiguous VRAM
 * (hipDeviceMallocContiguous: the largest translation fragments).  Free with sa_device_free. */
int sa_device_alloc(int64_t bytes, int32_t flags, void** out);
int sa_device_free(void* p);
/* Pitched asynchronous copy (hipMemcpy2DAsync, direction from the pointers): `height` rows of
 * `width` bytes, row r from src + r * spitch to dst + r * dpitch.  The pandas boundary's
 * pipeline copies a chunk's [cols x rows] output block into column-major host blocks of the
 * whole frame with one DMA per block (socceraction_amd/pipeline.py). */
int sa_copy2d_async(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                    int64_t height, void* stream);
/* Stream-ordering and timing events for device-local work: created with
 * hipEventDisableSystemFence, so recording one does not write back and invalidate the GPU's
 * caches the way a default event does (its system-scope release is what a host or peer reader
 * needs, not another stream of the same device: kernel boundaries already release to the
 * device).  timing = 0 also sets hipEventDisableTiming.  The bench step records its stream
 * forks / joins and per-kernel timings with these (torch.cuda.Event has no such flag). */
int sa_event_create(int32_t timing, void** ev);
int sa_event_destroy(void* ev);
int sa_event_record(void* ev, void* stream);
int sa_stream_wait_event(void* stream, void* ev);
int sa_event_synchronize(void* ev);
int sa_event_elapsed(void* start, void* end, float* ms);
/* Debug build (-DSA_DEBUG=1, libsocceraction_amd_debug.so): kernels check tile offsets,
 * column indices, segment cursors, LDS and grid-cell indices and record the first failure
 * instead of accessing out of bounds.  sa_debug_check() synchronises the device and returns
 * SA_EDATA with the source location in sa_last_error() if any check failed since the last
 * call (always SA_OK in the default build); sa_debug_enabled() tells the builds apart. */
int sa_debug_check(void);
/* Debug build only (SA_EINVAL otherwise): the next large-grid reordered solves have their last
 * workgroup leave at iteration `iteration` without arriving at the grid barrier, so the others
 * time out and the solve takes its barrier-timeout exit (SA_XT_PATH_TIMEOUT) -- the fallback a
 * GPU shared with another persistent grid takes.  -1 switches it off. */
int sa_debug_xt_solve_abort(int32_t iteration);
int sa_debug_enabled(void);

#ifdef __cplusplus
}
#endif
#endif /* SOCCERACTION_AMD_H */
