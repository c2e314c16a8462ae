// Decoder streaming-shape probe (round 5): y = norm * q * 2^-s over the Llama-400M arena
// (401 122 304 elements) for int8 (s <= 6) and int32 (s >= 7) payloads, one kernel per shape:
// V quads per thread, T threads per block, non-temporal or default loads and stores, and an
// XCD-grouped block order.  Interleaved rounds, median ms per launch; prints one line per shape.
// hipcc --offload-arch=gfx950 -O3 -o dec_shapes dec_shapes.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int W, int V, int T, bool NTL, bool NTS, bool XCD, bool ACC = false>
__global__ __launch_bounds__(T) void dec(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  uint32_t bid = blockIdx.x;
  if (XCD) {  // consecutive blocks of one XCD take consecutive ranges
    const uint32_t g = gridDim.x, per = g / 8;
    if (bid < per * 8) bid = (bid & 7) * per + (bid >> 3);
  }
  const int64_t base = (int64_t)bid * (V * T * 4);
  int32_t raw[V][W == 1 ? 1 : 4];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = min(base + 4 * ((int64_t)k * T + threadIdx.x), n - 4);
    if (W == 1) {
      const int32_t* p = reinterpret_cast<const int32_t*>(reinterpret_cast<const int8_t*>(q) + e);
      raw[k][0] = NTL ? __builtin_nontemporal_load(p) : *p;
    } else {
      const i32x4* p = reinterpret_cast<const i32x4*>(reinterpret_cast<const int32_t*>(q) + e);
      const i32x4 t = NTL ? __builtin_nontemporal_load(p) : *p;
      raw[k][0] = t[0]; raw[k][1] = t[1]; raw[k][2] = t[2]; raw[k][3] = t[3];
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)k * T + threadIdx.x);
    if (e >= n) continue;
    int32_t qi[4];
    if (W == 1) {
      qi[0] = (int8_t)(raw[k][0] & 0xff); qi[1] = (int8_t)((raw[k][0] >> 8) & 0xff);
      qi[2] = (int8_t)((raw[k][0] >> 16) & 0xff); qi[3] = (int8_t)((raw[k][0] >> 24) & 0xff);
    } else {
      qi[0] = raw[k][0]; qi[1] = raw[k][1]; qi[2] = raw[k][2]; qi[3] = raw[k][3];
    }
    f32x4 o;
    o[0] = __fmul_rn(__fmul_rn(norm, (float)qi[0]), inv);
    o[1] = __fmul_rn(__fmul_rn(norm, (float)qi[1]), inv);
    o[2] = __fmul_rn(__fmul_rn(norm, (float)qi[2]), inv);
    o[3] = __fmul_rn(__fmul_rn(norm, (float)qi[3]), inv);
    f32x4* p = reinterpret_cast<f32x4*>(y + e);
    if (ACC) {
      const f32x4 pv = __builtin_nontemporal_load(p);
      o[0] = __fadd_rn(pv[0], o[0]); o[1] = __fadd_rn(pv[1], o[1]); o[2] = __fadd_rn(pv[2], o[2]); o[3] = __fadd_rn(pv[3], o[3]);
    }
    if (NTS) __builtin_nontemporal_store(o, p); else *p = o;
  }
}

// Encoder-shaped stream: read V float4 per thread, write one int8 quad (or an int32 quad) per float4.
template <int W, int V, int T>
__global__ __launch_bounds__(T) void enc(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * (V * T * 4);
  f32x4 v[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = min(base + 4 * ((int64_t)k * T + threadIdx.x), n - 4);
    v[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(y + e));
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)k * T + threadIdx.x);
    if (e >= n) continue;
    int32_t l[4];
    for (int c = 0; c < 4; ++c) l[c] = (int32_t)__builtin_ceilf(__fmul_rn(v[k][c], norm) - inv);
    if (W == 1) {
      const uint32_t w = (uint32_t)(l[0] & 0xff) | (uint32_t)(l[1] & 0xff) << 8 | (uint32_t)(l[2] & 0xff) << 16 | (uint32_t)l[3] << 24;
      __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(const_cast<void*>(q)) + e));
    } else {
      const i32x4 o = {l[0], l[1], l[2], l[3]};
      __builtin_nontemporal_store(o, reinterpret_cast<i32x4*>(reinterpret_cast<int32_t*>(const_cast<void*>(q)) + e));
    }
  }
}

// The bracketed encoder's element map (4 Ki-element block, thread t of 256 owns rows
// b + 4 (k 256 + t), k = 0..3) cut into workgroups of WPB waves: workgroup i is waves
// (i mod (4 / WPB)) * WPB .. of block i / (4 / WPB).  WPB = 4 is today's pass.
template <int W, int WPB>
__global__ __launch_bounds__(64 * WPB) void encw(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  constexpr int per = 4 / WPB;
  const int64_t b = (int64_t)(blockIdx.x / per) * 4096;
  const int t = (blockIdx.x % per) * 64 * WPB + threadIdx.x;
  f32x4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = min(b + 4 * ((int64_t)k * 256 + t), n - 4);
    v[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(y + e));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = b + 4 * ((int64_t)k * 256 + t);
    if (e >= n) continue;
    int32_t l[4];
    for (int c = 0; c < 4; ++c) l[c] = (int32_t)__builtin_ceilf(__fmul_rn(v[k][c], norm) - inv);
    if (W == 1) {
      const uint32_t w = (uint32_t)(l[0] & 0xff) | (uint32_t)(l[1] & 0xff) << 8 | (uint32_t)(l[2] & 0xff) << 16 | (uint32_t)l[3] << 24;
      __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(const_cast<void*>(q)) + e));
    } else {
      const i32x4 o = {l[0], l[1], l[2], l[3]};
      __builtin_nontemporal_store(o, reinterpret_cast<i32x4*>(reinterpret_cast<int32_t*>(const_cast<void*>(q)) + e));
    }
  }
}

// Error-feedback shape (Top-K's streaming pass): r = r + x, V float4 of each per thread.
template <int V, int T>
__global__ __launch_bounds__(T) void efb(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * (V * T * 4);
  const float* x = reinterpret_cast<const float*>(q);
  f32x4 a[V], b[V];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = min(base + 4 * ((int64_t)k * T + threadIdx.x), n - 4);
    a[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + e));
    b[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(y + e));
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)k * T + threadIdx.x);
    if (e >= n) continue;
    f32x4 o = a[k] * norm + b[k];
    __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y + e));
  }
}

// Write-only stream (the Top-K decode's zero-filled tiles): V float4 stores per thread.
template <int V, int T>
__global__ __launch_bounds__(T) void wro(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * (V * T * 4);
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)k * T + threadIdx.x);
    if (e >= n) continue;
    const f32x4 o = {norm, 0.f, inv, 0.f};
    __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y + e));
  }
}

// Wave-contiguous layouts: wave w of the workgroup owns V consecutive 1 KiB pieces (lane l of
// store k at 4 (w 64 V + k 64 + l)) instead of pieces T x 16 bytes apart.
template <int V, int T>
__global__ __launch_bounds__(T) void wroc(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * (V * T * 4);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)w * 64 * V + k * 64 + l);
    if (e >= n) continue;
    const f32x4 o = {norm, 0.f, inv, 0.f};
    __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y + e));
  }
}
template <int W, int V, int T>
__global__ __launch_bounds__(T) void decc(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * (V * T * 4);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  int32_t raw[V][W == 1 ? 1 : 4];
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = min(base + 4 * ((int64_t)w * 64 * V + k * 64 + l), n - 4);
    if (W == 1) {
      raw[k][0] = *reinterpret_cast<const int32_t*>(reinterpret_cast<const int8_t*>(q) + e);
    } else {
      const i32x4 t = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(reinterpret_cast<const int32_t*>(q) + e));
      raw[k][0] = t[0]; raw[k][1] = t[1]; raw[k][2] = t[2]; raw[k][3] = t[3];
    }
  }
#pragma unroll
  for (int k = 0; k < V; ++k) {
    const int64_t e = base + 4 * ((int64_t)w * 64 * V + k * 64 + l);
    if (e >= n) continue;
    int32_t qi[4];
    if (W == 1) {
      qi[0] = (int8_t)(raw[k][0] & 0xff); qi[1] = (int8_t)((raw[k][0] >> 8) & 0xff);
      qi[2] = (int8_t)((raw[k][0] >> 16) & 0xff); qi[3] = (int8_t)((raw[k][0] >> 24) & 0xff);
    } else {
      qi[0] = raw[k][0]; qi[1] = raw[k][1]; qi[2] = raw[k][2]; qi[3] = raw[k][3];
    }
    f32x4 o;
    for (int c = 0; c < 4; ++c) o[c] = __fmul_rn(__fmul_rn(norm, (float)qi[c]), inv);
    __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y + e));
  }
}

// The encoder shape with its block's start read from a table first (the bracketed pass's item
// lookup before its loads): IND = 1 table load, 0 = arithmetic.
__device__ int64_t* g_btab;
template <int IND>
__global__ __launch_bounds__(256) void enci(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = IND ? reinterpret_cast<const int64_t* __restrict__>(g_btab)[blockIdx.x] : (int64_t)blockIdx.x * 4096;
  f32x4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = min(base + 4 * ((int64_t)k * 256 + threadIdx.x), n - 4);
    v[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(y + e));
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = base + 4 * ((int64_t)k * 256 + threadIdx.x);
    if (e >= n) continue;
    int32_t l[4];
    for (int c = 0; c < 4; ++c) l[c] = (int32_t)__builtin_ceilf(__fmul_rn(v[k][c], norm) - inv);
    const uint32_t w = (uint32_t)(l[0] & 0xff) | (uint32_t)(l[1] & 0xff) << 8 | (uint32_t)(l[2] & 0xff) << 16 | (uint32_t)l[3] << 24;
    __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(const_cast<void*>(q)) + e));
  }
}

// A looping tile writer: one workgroup of T threads per 64 Ki elements, one float4 per thread per
// iteration (T x 4 elements), a workgroup barrier between iterations (the tile decoder's LDS phases).
template <int T, bool BAR>
__global__ __launch_bounds__(T) void wrl(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 65536;
  for (int it = 0; it < 65536 / (4 * T); ++it) {
    const int64_t e = base + 4 * ((int64_t)it * T + threadIdx.x);
    if (e < n) {
      const f32x4 o = {norm, (float)it, inv, 0.f};
      __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y + e));
    }
    if (BAR) __syncthreads();
  }
}

// The same with the workgroups' chunks interleaved: iteration it of workgroup g writes chunk
// it * G + g (G workgroups), so the workgroups running together write neighbouring chunks.
template <int T, bool BAR>
__global__ __launch_bounds__(T) void wrs(const void* __restrict__ q, float* __restrict__ y, float norm, float inv, int64_t n) {
  const int64_t G = gridDim.x;
  for (int it = 0; it < 65536 / (4 * T); ++it) {
    const int64_t e = ((int64_t)it * G + blockIdx.x) * (4 * T) + 4 * threadIdx.x;
    if (e < n) {
      const f32x4 o = {norm, (float)it, inv, 0.f};
      __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(y + e));
    }
    if (BAR) __syncthreads();
  }
}

struct Shape {
  const char* name;
  void (*fn)(const void*, float*, float, float, int64_t);
  int blk_elems, threads;
  bool acc;
  int lds = 0;  // dynamic LDS bytes per workgroup: caps workgroups per CU (160 KiB / lds)
};

#define SH(W, V, T, L, S, X) Shape{"W" #W " V" #V " T" #T " ntl" #L " nts" #S " xcd" #X, \
                                   (void (*)(const void*, float*, float, float, int64_t))dec<W, V, T, L, S, X>, V * T * 4, T, false}
#define SHE(W, V, T) Shape{"ENC W" #W " V" #V " T" #T, \
                           (void (*)(const void*, float*, float, float, int64_t))enc<W, V, T>, V * T * 4, T, false}
#define SHW(W, WPB) Shape{"ENCW W" #W " wpb" #WPB, \
                           (void (*)(const void*, float*, float, float, int64_t))encw<W, WPB>, 1024 * WPB, 64 * WPB, false}
#define SHF(V, T) Shape{"EF V" #V " T" #T, \
                           (void (*)(const void*, float*, float, float, int64_t))efb<V, T>, V * T * 4, T, true}
#define SHWR(V, T) Shape{"WR V" #V " T" #T, \
                           (void (*)(const void*, float*, float, float, int64_t))wro<V, T>, V * T * 4, T, false}
#define SHWC(V, T) Shape{"WRC V" #V " T" #T, \
                           (void (*)(const void*, float*, float, float, int64_t))wroc<V, T>, V * T * 4, T, false}
#define SHDC(W, V, T) Shape{"DECC W" #W " V" #V " T" #T, \
                           (void (*)(const void*, float*, float, float, int64_t))decc<W, V, T>, V * T * 4, T, false}
#define SHI(I) Shape{"ENCI ind" #I, (void (*)(const void*, float*, float, float, int64_t))enci<I>, 4096, 256, false}
#define SHL(T, B) Shape{"WRL T" #T " bar" #B, \
                           (void (*)(const void*, float*, float, float, int64_t))wrl<T, B>, 65536, T, false}
#define SHS(T, B) Shape{"WRS T" #T " bar" #B, \
                           (void (*)(const void*, float*, float, float, int64_t))wrs<T, B>, 65536, T, false}
#define SHA(W, V, T) Shape{"ACC W" #W " V" #V " T" #T, \
                           (void (*)(const void*, float*, float, float, int64_t))dec<W, V, T, true, true, false, true>, V * T * 4, T, true}

int main(int argc, char** argv) {
  const int64_t n = 401122304;
  const int W = argc > 1 ? atoi(argv[1]) : 1;
  std::vector<Shape> shapes;
  if (argc > 2 && W == 300) {  // looping tile writers
    for (int lds : {0, 40960, 81920}) {
      for (Shape a : {SHWR(1, 256), SHL(256, true), SHS(256, true), SHS(256, false), SHS(512, true), SHS(1024, true)}) { a.lds = lds; shapes.push_back(a); }
    }
  } else if (argc > 2 && W == 200) {  // table-indirected block starts
    shapes = {SHI(0), SHI(1), SHE(1, 4, 256)};
  } else if (argc > 2 && W == 100) {  // wave-contiguous write-only
    for (int lds : {0, 24576, 40960}) {
      for (Shape a : {SHWR(1, 256), SHWR(8, 512), SHWC(8, 512), SHWC(4, 256), SHWC(8, 256), SHWC(16, 256)}) { a.lds = lds; shapes.push_back(a); }
    }
  } else if (argc > 2 && (W == 101 || W == 104)) {  // wave-contiguous decode
    const int w = W - 100;
    for (int lds : {0, 24576, 40960}) {
      for (Shape a : (w == 1 ? std::vector<Shape>{SH(1, 2, 256, 0, 1, 0), SH(1, 4, 256, 0, 1, 0), SHDC(1, 4, 256), SHDC(1, 2, 256), SHDC(1, 8, 256)}
                             : std::vector<Shape>{SH(4, 1, 256, 1, 1, 0), SH(4, 4, 256, 1, 1, 0), SHDC(4, 4, 256), SHDC(4, 2, 256), SHDC(4, 8, 256)})) {
        a.lds = lds; shapes.push_back(a);
      }
    }
  } else if (argc > 2 && W == 0) {  // write-only
    for (int lds : {0, 24576, 40960}) {
      for (Shape a : {SHWR(1, 256), SHWR(2, 256), SHWR(4, 256), SHWR(8, 256), SHWR(1, 128), SHWR(4, 512), SHWR(16, 512)}) { a.lds = lds; shapes.push_back(a); }
    }
  } else if (argc > 2 && W == 12) {  // the error-feedback shape (12 bytes per element)
    for (int lds : {0, 16384, 24576}) {
      for (Shape a : {SHF(1, 256), SHF(2, 256), SHF(1, 512), SHF(1, 128), SHF(2, 128)}) { a.lds = lds; shapes.push_back(a); }
    }
  } else if (argc > 2) {  // occupancy sweep of the encoder shapes
    for (int lds : {0, 16384, 24576, 32768, 40960}) {
      Shape a = W == 1 ? SHE(1, 4, 256) : SHE(4, 4, 256); a.lds = lds; shapes.push_back(a);
      Shape b = W == 1 ? SHE(1, 2, 256) : SHE(4, 1, 256); b.lds = lds; shapes.push_back(b);
    }
  } else if (W == 1) {
    shapes = {SH(1, 4, 256, 1, 1, 0), SH(1, 2, 256, 1, 1, 0), SH(1, 2, 128, 1, 1, 0), SH(1, 4, 128, 1, 1, 0),
              SH(1, 1, 512, 1, 1, 0), SH(1, 1, 1024, 1, 1, 0), SH(1, 2, 512, 1, 1, 0), SH(1, 2, 256, 0, 1, 0),
              SHA(1, 4, 256), SHA(1, 2, 256), SHA(1, 1, 256), SHA(1, 1, 512),
              SHE(1, 4, 256), SHE(1, 2, 256), SHE(1, 1, 256), SHE(1, 8, 256), SHE(1, 1, 512), SHW(1, 4), SHW(1, 2), SHW(1, 1)};
  } else {
    shapes = {SH(4, 4, 256, 1, 1, 0), SH(4, 1, 256, 1, 1, 0), SH(4, 1, 128, 1, 1, 0), SH(4, 2, 128, 1, 1, 0),
              SH(4, 1, 512, 1, 1, 0), SH(4, 1, 256, 1, 1, 1), SH(4, 1, 256, 0, 1, 0), SH(4, 1, 256, 1, 0, 0),
              SHA(4, 4, 256), SHA(4, 2, 256), SHA(4, 1, 256), SHA(4, 1, 512),
              SHE(4, 4, 256), SHE(4, 2, 256), SHE(4, 1, 256), SHE(4, 8, 256), SHE(4, 1, 512), SHW(4, 4), SHW(4, 2), SHW(4, 1)};
  }
  void* q; float* y;
  if (W == 200) {
    std::vector<int64_t> bt((n + 4095) / 4096);
    for (size_t i = 0; i < bt.size(); ++i) bt[i] = (int64_t)i * 4096;
    int64_t* d;
    CK(hipMalloc(&d, bt.size() * 8));
    CK(hipMemcpy(d, bt.data(), bt.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_btab), &d, sizeof(d)));
  }
  const int qb = W == 300 ? 1 : W == 200 ? 1 : W == 12 ? 4 : (W == 0 || W == 100) ? 1 : W > 100 ? W - 100 : W;
  CK(hipMalloc(&q, n * qb + 64));
  CK(hipMalloc(&y, n * 4 + 64));
  CK(hipMemset(q, 3, n * qb));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int reps = 20, rounds = 7;
  std::vector<std::vector<float>> ms(shapes.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < shapes.size(); ++i) {
      const Shape& s = shapes[i];
      const int grid = (int)((n + s.blk_elems - 1) / s.blk_elems);
      hipLaunchKernelGGL(s.fn, dim3(grid), dim3(s.threads), s.lds, 0, q, y, 1.5f, 0.125f, n);
      CK(hipEventRecord(a));
      for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(s.fn, dim3(grid), dim3(s.threads), s.lds, 0, q, y, 1.5f, 0.125f, n);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float t;
      CK(hipEventElapsedTime(&t, a, b));
      ms[i].push_back(t / reps);
    }
  }
  for (size_t i = 0; i < shapes.size(); ++i) {
    std::sort(ms[i].begin(), ms[i].end());
    const double med = ms[i][rounds / 2];
    const double bytes = W == 300 ? 4.0 * n : W == 200 ? 5.0 * n : (W == 0 || W == 100) ? 4.0 * n : W > 100 ? (double)n * (W - 100 + 4) : W == 12 ? 12.0 * n : (double)n * (W + (shapes[i].acc ? 8 : 4));
    char nm[96];
    snprintf(nm, sizeof nm, "%s lds%dK", shapes[i].name, shapes[i].lds / 1024);
    printf("%-36s median %.4f ms  min %.4f  %.2f TB/s\n", nm, med, ms[i][0], bytes / med / 1e9);
  }
  return 0;
}
