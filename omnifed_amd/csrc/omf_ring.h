// omf_ring.h — internal interface of the single-read QSGD encoder (omf_qsgd_ring.hip).
//
// Not part of the C ABI: the plan (omf_qsgd.hip) builds the work-item tables and calls
// omf::ring::launch.  DESIGN.md §3.1 describes the algorithm.
#pragma once

#include "omf_common.h"

namespace omf {
namespace ring {

// Work-item flags: a chunk publishes its partial sum of squares and/or quantises.
//   kPublish | kQuant  HOLD   read once: partial, keep the chunk on chip, quantise later
//   kPublish           NORM   partial only (first pass of a tensor too large to hold)
//   kQuant             QUANT  second pass of such a tensor: re-read and quantise
enum : int32_t { kPublish = 1, kQuant = 2 };

// 64 bytes = one scalar load: the tensor's fields ride along so the hot loops never make
// a second, dependent table read.
struct Item {
  int64_t begin, end;    // arena element range (one chunk of one tensor)
  int64_t tbegin, tn;    // the tensor's range
  int32_t tensor, flags, chunk, nchunks;
  int32_t gbase, pad[3];  // the tensor's first granule
};

struct Tensor {
  int64_t begin, n;
  int32_t nchunks, gbase;  // partial granules of this tensor: gran[gbase .. gbase + nchunks)
  int32_t pad[2];
};

struct Args {
  const float* x;
  const float* u;
  void* q;
  float* norm_out;
  const Item* items;
  const Tensor* tinfo;
  uint64_t* gran;  // {epoch << 32 | fp32 partial bits} per chunk
  uint32_t* err;
  int64_t n_items;
  float alpha;
  float levels;
  // PS fusion (omf_ps_apply_encode): divide != 0 -> the encoder's input is x / divisor
  // (IEEE, correctly rounded) instead of x * alpha, and xout (if set) receives it.
  float divisor;
  uint32_t divide;
  float* xout;
  uint32_t seed_lo, seed_hi, offset;
  uint32_t fmt;       // value format (omf_qsgd_dev.h kFmt*): rounding of norm and v / norm
  uint32_t round_in;  // fmt != F32 and alpha != 1: the weighted input is rounded to fmt
  uint32_t epoch;  // per-launch granule tag (never 0)
  uint64_t wait_ticks;      // bound of a norm wait (tunable: tests force the recompute fallback)
  uint64_t lds_wait_ticks;  // bound of an on-chip LDS hand-off wait (20 ms; expiry aborts)
  // test / experiment switches (omf_plan_set_debug, 0 in production): 1 = no norm wait
  // (norm := 1), 2 = no quantisation, 4 = time phases, 8 = slots never marked loaded
  uint32_t dbg;
  unsigned long long* prof;  // dbg & 4: per-phase cycle totals (omf_plan_ring_profile)
};

struct Config {
  int rows;     // rows of 1024 elements per chunk
  int slots;    // LDS ring slots (each one chunk)
  int loaders;  // loader waves of the 16 (the rest quantise)
  int dbuf;     // loaders prefetch two chunks ahead
  int kind = 0;  // 0: LDS ring (qsgd_encode_pc); 1: register-resident (qsgd_encode_rr, slots =
                 // register buffers per thread; the plan packs single-read tensors in one row)
};

int num_configs();
Config config(int cfg);
inline int64_t chunk_elems(const Config& c) { return (int64_t)c.rows * 1024; }
// Co-resident workgroups of one launch on `device` (occupancy x CUs, LDS-capped).
int grid_size(int cfg, int device);
// 0 on success; caller checks hipGetLastError.
int launch(int cfg, int width, bool has_u, const Args& a, int grid, hipStream_t stream);

}  // namespace ring
}  // namespace omf
