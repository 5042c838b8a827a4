// Shared device helpers for libddq_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

// A/B timing experiments only (make variant DEFS=-DDDQ_AB_SKIP=..., tools/ab):
// work that returns at once -- slab-reduce launch roles (1 fc4 apply tiles,
// 2 slab units, 4 head sums, 8 prefetch); conv2 forward phases (16 the tap
// loop, 32 the epilogue stores, 64 the patch staging).  0 in the product build.
#ifndef DDQ_AB_SKIP
#define DDQ_AB_SKIP 0
#endif
// A/B: force a conv tile-menu entry (kernels.hip pick_tile), -1 = the cost model's
#ifndef DDQ_AB_TILE_C1F
#define DDQ_AB_TILE_C1F -1
#endif
#ifndef DDQ_AB_TILE_C2F
#define DDQ_AB_TILE_C2F -1
#endif
#ifndef DDQ_AB_TILE_C3F
#define DDQ_AB_TILE_C3F -1
#endif
#ifndef DDQ_AB_TILE_C3D
#define DDQ_AB_TILE_C3D -1
#endif
#ifndef DDQ_AB_TILE_C2D
#define DDQ_AB_TILE_C2D -1
#endif
// A/B: workgroups the conv2 / conv3 weight gradients aim at (kernels.hip
// wgrad_splits_for: fewer = fewer, larger slabs)
#ifndef DDQ_AB_WG_TARGET2
#define DDQ_AB_WG_TARGET2 256   // 24 slabs at 64x64 B=32: pair 28.4 -> 27.7 us, 6098 -> 6165 updates/s A/B
#endif
#ifndef DDQ_AB_WG_TARGET3
#define DDQ_AB_WG_TARGET3 256   // 40 slabs at 64x64 B=32: pair 30.0 -> 28.2 us, reduce 21.9 -> 19.2
#endif
// A/B: the conv1 weight gradient's largest band height (kernels.hip wgrad1_band)
#ifndef DDQ_AB_W1BAND
#define DDQ_AB_W1BAND 8
#endif
// A/B: waves of a conv1 weight-gradient workgroup (wgrads.h launch_wgrad1s_w)
#ifndef DDQ_AB_W1NW
#define DDQ_AB_W1NW 4
#endif
// A/B: k per fc4-forward split (fc.h kFc4KLen; the head sums K / kFc4KLen partials);
// measured: 64 -> head 6.6 -> 8.4 us, 256 -> fc4 forward 6.0 -> 8.7 us (128 kept)
#ifndef DDQ_AB_FC4_KLEN
#define DDQ_AB_FC4_KLEN 128
#endif
// A/B: the conv1 weight gradient stages one conv row of a pooled row at a time
// (3 LDS planes per wave instead of 6: two workgroups per CU); measured:
// conv1 weight gradient 14.2 -> 15.6 us (256 workgroups never pair on a CU)
#ifndef DDQ_AB_W1SEQ
#define DDQ_AB_W1SEQ 0
#endif
// the slab-reduce launch dispatches its 8 head-sum blocks right after the
// prefetch blocks instead of last (kernels.hip wgrad_reduce_kernel); 1 in the
// product build: reduce 19.4 -> 16.4 us, 6108 -> 6250 updates/s (same-box A/B)
#ifndef DDQ_REDUCE_HEAD_FIRST
#define DDQ_REDUCE_HEAD_FIRST 1
#endif
// A/B (with DDQ_REDUCE_HEAD_FIRST): the 8 head-sum blocks dispatched before the
// next step's draw + gather blocks; measured 6310 -> 6245 updates/s (rejected)
#ifndef DDQ_REDUCE_PF_AFTER_HEAD
#define DDQ_REDUCE_PF_AFTER_HEAD 0
#endif
// A/B (with DDQ_REDUCE_HEAD_FIRST): the slab units dispatched before the fused
// fc4 apply tiles; measured: reduce 16.6 -> 22.6 us, 6254 -> 6012 updates/s (rejected)
#ifndef DDQ_REDUCE_SLABS_FIRST
#define DDQ_REDUCE_SLABS_FIRST 0
#endif
// A/B: static s_setprio 1 for the second half of the waves of the split-conv
// and weight-gradient-pair workgroups (MI355X_MICROARCH.md item 4); measured
// 6314 -> 6327 updates/s over two A/B pairs, kernel times unchanged (not adopted)
#ifndef DDQ_AB_SETPRIO
#define DDQ_AB_SETPRIO 0
#endif
// conflict-free LDS stores of 32-channel weight rows and patch pixels
// (split.h SplitWStage::row); 1 in the product build (timing-neutral:
// conv2 forward 30.4 -> 30.2 us, within the A/B's noise)
#ifndef DDQ_LDS_ROWPERM
#define DDQ_LDS_ROWPERM 1
#endif
// A/B: conv3 forward on 8 x 16 tiles, 16 waves; measured 11.2 -> 14.6 us
#ifndef DDQ_AB_C3F_WIDE
#define DDQ_AB_C3F_WIDE 0
#endif
// fc4 data gradient: the two 16-column blocks of a 128-byte W4 line on one XCD;
// 1 in the product build: 7.1 -> 6.5 us
#ifndef DDQ_FC4BWD_XCD
#define DDQ_FC4BWD_XCD 1
#endif
// Measured and rejected (same-box A/B, 64x64 B=32, rocprofv3 averages; 0 in
// the product build, where their kernels are not even instantiated):
//  DDQ_CONV2_PIPE  conv2 forward as the persistent pipelined kernel (split.h
//                  split_conv_pipe_body, 8 x 16 tiles, 8 waves): 30.8 -> 52.0 us
//  DDQ_C2D_PIPE    conv2 data gradient likewise (two 32-channel chunks): 20.5 -> 36.5 us
//  DDQ_CONV1_PIPE  conv1 forward likewise (split_conv1_pipe_kernel): 12.2 -> 12.9 us
//  DDQ_FC4_CHAIN   fc4 forward + head + fc4 data gradient as one launch with
//                  intra-launch counter hand-offs (fc4_chain_kernel): 19.8 -> 31.2 us
//  DDQ_FA_IN_PAIR  the fused fc4-weight apply blocks interleaved into the conv2 / conv3
//                  weight-gradient launch (wgrads_pair_fa_kernel): reduce 19.2 -> 12.2 us
//                  but the pair 28.4 -> 44.4 us (6098 -> 5797 updates/s)
#ifndef DDQ_CONV2_PIPE
#define DDQ_CONV2_PIPE 0
#endif
#ifndef DDQ_C2D_PIPE
#define DDQ_C2D_PIPE 0
#endif
#ifndef DDQ_CONV1_PIPE
#define DDQ_CONV1_PIPE 0
#endif
#ifndef DDQ_FC4_CHAIN
#define DDQ_FC4_CHAIN 0
#endif
#ifndef DDQ_FA_IN_PAIR
#define DDQ_FA_IN_PAIR 0
#endif

namespace ddq {

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kActions = 4;        // barista/constants.py:8
constexpr int kFrames = 4;         // expgain.py:9
constexpr int kFc4 = 512;          // train_val.prototxt:169

// Division by a runtime constant (multiply-high + shift), exact for
// 0 <= n < 2^31 (Granlund-Montgomery / Hacker's Delight round-up method).
struct FastDiv {
  uint32_t d, mul, shr;
  FastDiv() = default;
  __host__ explicit FastDiv(uint32_t divisor) : d(divisor) {
    if (divisor == 1) { mul = 0; shr = 0; return; }
    uint32_t l = 0;
    while ((1ull << l) < divisor) ++l;
    uint64_t m = ((1ull << 32) * ((1ull << l) - divisor)) / divisor + 1;
    mul = (uint32_t)m;
    shr = l - 1;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    if (d == 1) return n;
    uint32_t t = __umulhi(n, mul);
    return (t + ((n - t) >> 1)) >> shr;
  }
  __device__ __forceinline__ void divmod(uint32_t n, uint32_t& q, uint32_t& r) const {
    q = div(n);
    r = n - q * d;
  }
};

__device__ __forceinline__ float4 f4(float a, float b, float c, float d) {
  return make_float4(a, b, c, d);
}
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

}  // namespace ddq
