// ie_lean.hip — k_lean: interpolate_inserts (py:497-541 / rust-project/src/interp.rs:31-89) for the
// common string shape, into a views output (include/ie_amd.h ie_interpolate_device_views).
//
// One WAVE per tile of 64 consecutive strings (a 64-lane workgroup, persistent over the batch):
// no workgroup barrier, no look-back, no LDS output stage, so a tile holds 7.7 KB of LDS and few
// registers, and about twice as many strings are in flight per CU as in k_resolve. Per tile:
//   1. the tile's bytes (<= 6 KB) are loaded coalesced into the wave's LDS stage and every 16-byte
//      chunk is classified ('{' / '}' masks, '\' and 0xE3 bits) from the registers they came in;
//   2. each lane parses its string into chains (parse_chains, ie_bytes.h: the chain evaluator's
//      shape) and resolves its <= 3 chains level by level, innermost first, keys assembled in
//      registers (one pilot and one entry read per level, all chains of the wave in flight);
//   3. a wave scan of the output lengths, one atomic claim on one of R cursor shards: shard r owns
//      the stripes r, r + R, r + 2R, ... of S bytes of the output, so that 156k claims do not
//      serialize on one word; a string whose range would cross a stripe boundary claims again;
//   4. every lane stores its own string: template runs from the stage, value texts from the table,
//      with 16-byte stores (a piece's overrun is overwritten by the same lane's next piece; the
//      last piece of a string is stored exactly).
// Anything outside the shape (a string past the stage, a whole-string pair, a miss, a non-inert or
// unspliceable value, a long key or text) is listed for the fallback: k_resolve on the listed
// subset (exact evaluator, literal path), whose tiles claim after the stripes (W.cursor is set to
// their extent). Every string k_lean commits equals the chain evaluator's result.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_bytes.h"
#include "ie_device.h"
#include "ie_kernels.h"

#ifndef IE_LEAN_WAVES
#define IE_LEAN_WAVES 4
#endif

namespace ie {
namespace lean {

constexpr uint32_t kW = 64;             // strings per wave (its own stage, parse and lookups)
constexpr uint32_t kWaves = 4;          // waves per tile: one output claim per 256 strings
constexpr uint32_t kTile = kW * kWaves;
constexpr uint32_t kSpanChunks = 384;   // the stage: 6 KB of the tile's bytes
constexpr int kLV = kSpanChunks / kW;   // chunk loads per lane
constexpr uint32_t kOddWords = kSpanChunks / 32 + 2;
constexpr uint32_t kMaxArenaText = 256; // longer top-level texts: the fallback
constexpr uint32_t kShardStride = 16;   // u64 words between cursor shards (128 B)

typedef __attribute__((address_space(1))) u32x4_ua g_v4u;
typedef __attribute__((address_space(1))) u64_ua g_u64u;
typedef __attribute__((address_space(1))) u32_ua g_u32u;
typedef __attribute__((address_space(1))) u16_ua g_u16u;

#ifndef IE_LEAN_NT
#define IE_LEAN_NT 0
#endif
__device__ __forceinline__ void gst16u(uint8_t* p, u32x4 v) {
#if IE_LEAN_NT
  __builtin_nontemporal_store(v, (g_v4u*)p);
#else
  *(g_v4u*)p = v;
#endif
}
__device__ __forceinline__ u32x4 gld16u(const uint8_t* p) { return *(const g_v4u*)p; }

// the first len (< 16) bytes of v to p (any alignment)
__device__ __forceinline__ void gst_part(uint8_t* p, u32x4 v, uint32_t len) {
  uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  const uint64_t hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  if (len & 8) {
    *(g_u64u*)p = lo;
    lo = hi;
    p += 8;
  }
  if (len & 4) {
    *(g_u32u*)p = (uint32_t)lo;
    lo >>= 32;
    p += 4;
  }
  if (len & 2) {
    *(g_u16u*)p = (uint16_t)lo;
    lo >>= 16;
    p += 2;
  }
  if (len & 1) *(__attribute__((address_space(1))) uint8_t*)p = (uint8_t)lo;
}

// chunk_classify (ie_bytes.h) on a chunk in registers
__device__ __forceinline__ uint32_t classify_regs(uint4 v, bool& odd, bool& esc) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t op = 0, cl = 0, od = 0, bs = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = w[k];
    const uint32_t x7 = x & 0x7F7F7F7Fu;
    const uint32_t no = ((x7 ^ 0x7B7B7B7Bu) + 0x7F7F7F7Fu) | x;
    const uint32_t nc = ((x7 ^ 0x7D7D7D7Du) + 0x7F7F7F7Fu) | x;
    const uint32_t nb = ((x7 ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu) | x;
    const uint32_t ne = ((x7 ^ 0x63636363u) + 0x7F7F7F7Fu) | ~x;
    od |= ~ne;
    bs |= ~nb;
    op |= nib(~no) << (4 * k);
    cl |= nib(~nc) << (4 * k);
  }
  odd = (od & 0x80808080u) != 0;
  esc = (bs & 0x80808080u) != 0;
  return op | (cl << 16);
}

// lane-to-lane LDS exchange inside one wave (no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave reductions and scans on DPP row shifts plus scalar read-lanes (no ds_bpermute: its lane
// indices are loop invariants the compiler keeps live across the tile loop, and spills)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {  // lanes shifted in from outside the row read 0
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t rdlane(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
// max over the wave (uniform result)
__device__ __forceinline__ uint32_t wave_umax(uint32_t x) {
  x = umax32(x, dpp0<0x111>(x));  // row_shr:1
  x = umax32(x, dpp0<0x112>(x));  // row_shr:2
  x = umax32(x, dpp0<0x114>(x));  // row_shr:4
  x = umax32(x, dpp0<0x118>(x));  // row_shr:8 (lane 15 of each row: the row's max)
  return umax32(umax32(rdlane(x, 15), rdlane(x, 31)), umax32(rdlane(x, 47), rdlane(x, 63)));
}
// exclusive prefix sum over the wave; total = the wave's sum (uniform)
__device__ __forceinline__ uint32_t wave_scan_excl(uint32_t v, uint32_t& total) {
  uint32_t x = v;
  x += dpp0<0x111>(x);
  x += dpp0<0x112>(x);
  x += dpp0<0x114>(x);
  x += dpp0<0x118>(x);  // inclusive within each row of 16 lanes
  const uint32_t r0 = rdlane(x, 15), r1 = rdlane(x, 31), r2 = rdlane(x, 47), r3 = rdlane(x, 63);
  const uint32_t row = lane_id() >> 4;
  x += row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r0 + r1 : r0 + r1 + r2;
  total = r0 + r1 + r2 + r3;
  return x - v;
}
__device__ __forceinline__ uint64_t lane0_u64(uint64_t v) {
  return ((uint64_t)rdlane((uint32_t)(v >> 32), 0) << 32) | rdlane((uint32_t)v, 0);
}

// value kinds of a chain's result (as k_resolve's descriptors)
enum : uint32_t { kValArena = 1, kValEntry = 3 };

// Level-by-level resolution of (up to) two chains of this lane's string, innermost first: the key of
// a level is A | T | B (template before the child, the child's splice text, template after it; a
// leaf: A only), assembled in registers and looked up with one pilot and one entry read, both
// chains' reads in flight together (and every lane's). rk / rs: the top level's value (kind << 30 |
// text length; entry index or arena offset); rej: a condition the chain evaluator cannot commit
// (long key or text, a miss, a non-inert or unspliceable value): the string takes the fallback.
template <bool MULTI>
__device__ __forceinline__ void resolve2(const DevTable& T, const lds_u8* s, uint32_t tb, const Ev& Om, const Ev& Cm,
                                         bool on0, uint32_t cr0, uint32_t dp0, bool on1, uint32_t cr1, uint32_t dp1,
                                         uint32_t& rk0, uint32_t& rs0, uint32_t& rk1, uint32_t& rs1, bool& rej) {
  constexpr int NJ = 2;
  const uint32_t crec[NJ] = {cr0, cr1}, cdep[NJ] = {on0 ? dp0 : 0u, on1 ? dp1 : 0u};
  uint32_t rk[NJ] = {0u, 0u}, rs[NJ] = {0u, 0u};
  uint32_t co[NJ] = {0u, 0u}, cl[NJ] = {0u, 0u}, ctl[NJ] = {0u, 0u};
  u32x4 ct[NJ] = {u32x4{0, 0, 0, 0}, u32x4{0, 0, 0, 0}};
  bool done[NJ] = {!on0, !on1};
  const uint32_t rounds = wave_umax(cdep[0] > cdep[1] ? cdep[0] : cdep[1]);
  for (uint32_t r = 0; r < rounds; r++) {
    bool on[NJ], top[NJ];
    uint32_t open[NJ], close[NJ], klen[NJ], slot[NJ];
    u32x4 kw[NJ];
    uint64_t h[NJ];
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      on[q] = !done[q] && r < cdep[q];
      top[q] = r + 1 == cdep[q];
      // level r: the innermost pair in round 0, the outermost in the last; a middle level is the
      // open before the previous level's and the close after it
      uint32_t o = r == 0 ? (crec[q] >> 16) & 0xFFu : top[q] ? crec[q] & 0xFFu : 0u;
      uint32_t c = r == 0 ? (crec[q] >> 8) & 0xFFu : top[q] ? crec[q] >> 24 : 0u;
      if (on[q] && r != 0 && !top[q]) {
        o = ev_last(ev_below(Om, co[q]));
        c = ev_first(ev_from(Cm, cl[q] + 1u));
      }
      open[q] = on[q] ? o : 0u;
      close[q] = on[q] ? c : 0u;
      const uint32_t la = on[q] ? (r == 0 ? close[q] : co[q]) - open[q] - 1u : 0u;
      const uint32_t lb = on[q] && r != 0 ? close[q] - cl[q] - 1u : 0u;
      klen[q] = la + (r != 0 ? ctl[q] + lb : 0u);
      if (on[q] && klen[q] > kInlineKey) {  // a key longer than the entry's inline copy
        on[q] = false;
        done[q] = true;
        rej = true;
      }
      u32x4 k = keep_bytes(ld16a(s + open[q] + 1u), la);
      if (r != 0) {
        const u32x4 t = shl_bytes(ct[q], la);
        const u32x4 b = shl_bytes(keep_bytes(ld16a(s + cl[q] + 1u), lb), la + ctl[q]);
        k = u32x4{k.x | t.x | b.x, k.y | t.y | b.y, k.z | t.z | b.z, k.w | t.w | b.w};
      }
      kw[q] = keep_bytes(k, klen[q]);
      uint64_t hh = hash_init(klen[q], T.seed, tb);
      if (klen[q] > 0u) hh = hash_word(hh, kw[q].x);
      if (klen[q] > 4u) hh = hash_word(hh, kw[q].y);
      if (klen[q] > 8u) hh = hash_word(hh, kw[q].z);
      if (klen[q] > 12u) hh = hash_word(hh, kw[q].w);
      h[q] = hh;
    }
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      const uint32_t pilot = on[q] ? (uint32_t)gld(T.pilots + ph_group(h[q], T.nb)) : 0u;
      slot[q] = on[q] ? ph_slot(h[q], pilot, T.m) : 0u;
    }
    uint4 e0[NJ], e1[NJ], e2[NJ];
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      if (__any(on[q])) {
        const uint4* e = (const uint4*)(T.entries + slot[q]);
        e0[q] = gld4(e);
        e1[q] = gld4(e + 1);
        e2[q] = gld4(e + 2);
      }
    }
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      if (!__any(on[q])) continue;
      const bool hit = on[q] && (entry_head_ok(e0[q], klen[q], tb) & (e1[q].x == kw[q].x) & (e1[q].y == kw[q].y) &
                                 (e1[q].z == kw[q].z) & (e1[q].w == kw[q].w));
      const uint32_t flags = e0[q].z, tlen = e0[q].y;
      // only hits on inert, spliceable values commit here (then every evaluation order gives the
      // reference's bytes); misses and the rest take the fallback, which keeps the error order
      const bool good = hit && (flags & EF_SPLICE_OK) && (flags & EF_INERT);
      if (on[q] && !good) {
        done[q] = true;
        rej = true;
      }
      if (on[q] && good && !top[q]) {  // an inner level: its text goes into the parent's key
        if (tlen > kInlineKey) {
          done[q] = true;
          rej = true;
        }
        ct[q] = u32x4{e2[q].x, e2[q].y, e2[q].z, e2[q].w};
        ctl[q] = tlen;
        co[q] = open[q];
        cl[q] = close[q];
      }
      if (on[q] && good && top[q]) {
        const bool inl = tlen <= kInlineText;
        if (!inl && tlen > kMaxArenaText) rej = true;
        rk[q] = ((inl ? kValEntry : kValArena) << 30) | tlen;
        rs[q] = inl ? slot[q] : e0[q].w;
        done[q] = true;
      }
    }
  }
  rk0 = rk[0], rs0 = rs[0], rk1 = rk[1], rs1 = rs[1];
}

template <bool MULTI>
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(IE_LEAN_WAVES))) void k_lean(Batch B, Work W, DevTable T, uint8_t* out,
                                                                                               uint64_t cap) {
  __shared__ __attribute__((aligned(16))) uint8_t s_stage_all[kWaves][kSpanChunks * 16 + 48];
  __shared__ uint32_t s_cm_all[kWaves][kSpanChunks + 12];
  __shared__ uint32_t s_odd_all[kWaves][kOddWords], s_esc_all[kWaves][kOddWords];
  // the claim's words, double-buffered by tile parity (a wave may run into the next tile's claim
  // while another still reads this one's)
  __shared__ uint32_t s_wt[2][kWaves];
  __shared__ uint64_t s_base[2];
  const uint32_t lane = lane_id(), wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint8_t* const s_stage = s_stage_all[wave];
  uint32_t* const s_cm = s_cm_all[wave];
  uint32_t* const s_odd = s_odd_all[wave];
  uint32_t* const s_esc = s_esc_all[wave];
  if (lane < kOddWords - 2 * kLV) s_odd[2 * kLV + lane] = s_esc[2 * kLV + lane] = 0u;
  const uint64_t ntiles = (B.n + kTile - 1) / kTile;
  const uint32_t shard = blockIdx.x & (W.n_shards - 1u);
  unsigned long long* const ctr = (unsigned long long*)(W.shards + (uint64_t)shard * kShardStride);
  const uint32_t slog = W.stripe_log2, R = W.n_shards;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // diagnostic stamps (IE_DEBUG_STAMPS, 100 MHz s_memrealtime): the tile's row of 16 words, four
    // per wave: start, resolved, claimed, stored
    uint64_t* const stamp = W.stamps && lane == 0 ? W.stamps + tile * 16 + 4 * wave : nullptr;
    if (stamp) stamp[0] = __builtin_amdgcn_s_memrealtime();
    // ---- 1. geometry, stage, classification (each wave its own 64 strings) ----
    const uint64_t i = tile * kTile + threadIdx.x;
    const bool valid = i < B.n;
    uint64_t so = 0, sn = 0;
    if (valid) {
      so = gld(B.in_off + i);
      sn = B.in_len ? (uint64_t)gld(B.in_len + i) : gld(B.in_off + i + 1) - so;
    }
    const uint64_t lo = lane0_u64(so);
    const bool after = valid && so >= lo;  // (a views input may place a string before lane 0's)
    const uint64_t rel = after ? so + sn - lo : 0u;  // the wave's span past lo (beyond 4 GB: clamped)
    const uint64_t hi = lo + wave_umax(rel < 0xFFFFFFFFull ? (uint32_t)rel : 0xFFFFFFFFu);
    const uintptr_t plo = (uintptr_t)(B.bytes + lo);
    const uint32_t sh = (uint32_t)(plo & 15);
    const uint4* src = (const uint4*)(plo - sh);  // an aligned chunk never crosses a page
    const uint64_t need = ((uint64_t)sh + (hi - lo) + 15) >> 4;
    const uint32_t nv = (hi == lo && !after) ? 0u : need < kSpanChunks ? (uint32_t)need : kSpanChunks;
    uint4 v[kLV];
#pragma unroll
    for (int k = 0; k < kLV; k++) {
      const uint32_t c = lane + (uint32_t)k * kW;
      if (c < nv) v[k] = gld4s(src + c);
    }
#pragma unroll
    for (int k = 0; k < kLV; k++) {
      const uint32_t c = lane + (uint32_t)k * kW;
      bool odd = false, esc = false;
      if (c < nv) {
        ((uint4*)s_stage)[c] = v[k];
        s_cm[c] = classify_regs(v[k], odd, esc);
      }
      const uint64_t ob = __ballot(odd), eb = __ballot(esc);
      if (lane == 0) {
        s_odd[2 * k] = (uint32_t)ob, s_odd[2 * k + 1] = (uint32_t)(ob >> 32);
        s_esc[2 * k] = (uint32_t)eb, s_esc[2 * k + 1] = (uint32_t)(eb >> 32);
      }
    }
    if (lane < 12) s_cm[nv + lane] = 0u;  // the event windows read past the last chunk
    wave_sync();

    // ---- 2. chains: parse, then resolve level by level ----
    const uint32_t p0 = sh + (uint32_t)(so - lo);
    const bool staged = after && sn < 0xFFFF0000ull && (uint64_t)p0 + sn <= 16ull * nv;
    const uint32_t n32 = (uint32_t)sn;
    const uint32_t tb = (MULTI && valid) ? gld(B.table_id + i) : 0u;
    uint32_t crec[kMaxTop], cdep[kMaxTop], nch = 0, maxd = 0;
    Ev Om, Cm;
    bool whole1;  // (a whole-string '{key}': k_resolve's chain jobs take it, here the fallback)
    bool ok = parse_chains((const lds_u8*)s_stage, staged ? p0 : 0u, staged ? n32 : 0u, (const lds_u32*)s_cm,
                           (const lds_u32*)s_odd, (const lds_u32*)s_esc, staged, crec, cdep, nch, Om, Cm, maxd,
                           whole1);
    // (long templates with flat pairs have wide chain records: k_resolve's chain jobs take them;
    // a long brace-free string is copied here)
    ok = ok && !whole1 && (n32 <= kChainMax || nch == 0u);
    const lds_u8* const s = (const lds_u8*)s_stage + (staged ? p0 : 0u);
    uint32_t rk[kMaxTop], rs[kMaxTop];  // per chain: value kind << 30 | text length; entry / arena offset
    bool rej = false;
    // chains 0 and 1 together; chain 2 (rare) in a second pass, so that the registers hold two
    // chains' lookups in flight, not three
    resolve2<MULTI>(T, s, tb, Om, Cm, ok && nch > 0u, crec[0], cdep[0], ok && nch > 1u, crec[1], cdep[1], rk[0], rs[0],
                    rk[1], rs[1], rej);
    rk[2] = rs[2] = 0u;
    if (__any(ok && nch > 2u)) {
      uint32_t rk_x, rs_x;
      resolve2<MULTI>(T, s, tb, Om, Cm, ok && nch > 2u, crec[2], cdep[2], false, 0u, 0u, rk[2], rs[2], rk_x, rs_x, rej);
    }
    const bool fast = ok && !rej && staged;
    if (stamp) stamp[1] = __builtin_amdgcn_s_memrealtime();
    uint32_t olen = 0;
    if (fast) {
      uint32_t span = 0, vsum = 0;
#pragma unroll
      for (int q = 0; q < kMaxTop; q++) {
        if ((uint32_t)q < nch) {
          span += (crec[q] >> 24) - (crec[q] & 0xFFu) + 1u;
          vsum += rk[q] & ((1u << 30) - 1u);
        }
      }
      olen = n32 - span + vsum;
    }

    // ---- 3. the fallback list; the wave's output range ----
    const bool dfr = valid && !fast;
    const uint64_t dm = __ballot(dfr);
    if (dm) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(W.udefer_count, (uint32_t)__popcll(dm));
      base = rdlane(base, 0);
      if (dfr) W.udefer_list[base + (uint32_t)__popcll(dm & ((1ull << lane) - 1ull))] = (uint32_t)i;
    }
    uint32_t total;
    const uint32_t local = wave_scan_excl(fast ? olen : 0u, total);
    // the tile's output range: one claim for its four waves
    const uint32_t par = (uint32_t)(tile / gridDim.x) & 1u;
    if (lane == 0) s_wt[par][wave] = total;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t t = s_wt[par][0] + s_wt[par][1] + s_wt[par][2] + s_wt[par][3];
      s_base[par] = t ? atomicAdd(ctr, (unsigned long long)t) : 0ull;
    }
    // the texts of values 0 and 1 (inline ones from their entries; L2-warm) while the claim is in
    // flight; value 2's (rare) when it is stored
    u32x4 ta[2], tc[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const bool need_t = fast && (uint32_t)q < nch && (rk[q] >> 30) == kValEntry;
      ta[q] = tc[q] = u32x4{0, 0, 0, 0};
      if (__any(need_t)) {
        const u32x4* tp = (const u32x4*)(T.entries + (need_t ? rs[q] : 0u)) + 2;
        ta[q] = gld(tp);
        tc[q] = gld(tp + 1);
        tc[q].w = 0u;
      }
    }
    __syncthreads();
    if (stamp) stamp[2] = __builtin_amdgcn_s_memrealtime();
    uint64_t vv = s_base[par] + local;
#pragma unroll
    for (uint32_t w = 0; w < kWaves - 1; w++) vv += w < wave ? s_wt[par][w] : 0u;
    bool mine = fast;
    // a range that would cross a stripe boundary claims again (rare: one string per stripe)
    bool strad = fast && olen && ((vv >> slog) != ((vv + olen - 1u) >> slog));
    for (int attempt = 0; attempt < 4 && __any(strad); attempt++) {
      if (strad) {
        vv = atomicAdd(ctr, (unsigned long long)olen);
        strad = (vv >> slog) != ((vv + olen - 1u) >> slog);
      }
    }
    if (strad) {  // (never seen) the fallback writes it after all
      mine = false;
      const uint32_t b2 = atomicAdd(W.udefer_count, 1u);
      W.udefer_list[b2] = (uint32_t)i;
    }
    const uint64_t phys = ((((vv >> slog) * (uint64_t)R) + shard) << slog) | (vv & ((1ull << slog) - 1ull));
    if (mine) {
      gsts(B.out_off + i, phys);
      gsts(B.out_len + i, olen);
      gsts(B.status + i, (uint8_t)IE_OK_STR);
    }

    // ---- 4. this lane's bytes: template runs from the stage, values from the table ----
    if (mine && olen && phys + olen <= cap) {
      uint8_t* const dst = out + phys;
      // 16 bytes of a piece at output position p (nb of them the piece's): a full store while it ends
      // inside the string (the overrun is rewritten by this lane's next piece, in program order),
      // else exactly the piece's bytes (never past the string: the next string is another lane's)
      auto put = [&](u32x4 val, uint32_t p, uint32_t nb) {
        if (p + 16u <= olen) gst16u(dst + p, val);
        else gst_part(dst + p, val, nb < 16u ? nb : 16u);
      };
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j <= kMaxTop; j++) {
        const uint32_t t_lo = j == 0 ? 0u : (crec[j - 1] >> 24) + 1u;
        const uint32_t t_hi = (uint32_t)j < nch ? (crec[j] & 0xFFu) : n32;
        const uint32_t tl = (uint32_t)j <= nch ? t_hi - t_lo : 0u;
        for (uint32_t k = 0; k < tl; k += 16u) put(ld16a(s + t_lo + k), w + k, tl - k);
        w += tl;
        if (j == kMaxTop || (uint32_t)j >= nch) continue;
        const uint32_t len = rk[j] & ((1u << 30) - 1u);
        if ((rk[j] >> 30) == kValEntry) {
          u32x4 a, b;
          if (j < 2) {
            a = ta[j], b = tc[j];
          } else {
            const u32x4* tp = (const u32x4*)(T.entries + rs[j]) + 2;
            a = gld(tp), b = gld(tp + 1);
          }
          if (len) put(a, w, len);
          if (len > 16u) put(b, w + 16u, len - 16u);
        } else {
          const uint8_t* const ap = T.arena + rs[j];
          for (uint32_t k = 0; k < len; k += 16u) put(gld16u(ap + k), w + k, len - k);
        }
        w += len;
      }
    }
    if (stamp) stamp[3] = __builtin_amdgcn_s_memrealtime();
  }
}

// After k_lean: the stripes' extent becomes the fallback's cursor (its tiles claim after it)
__global__ void k_lean_finish(Work W) {
  const uint32_t lane = threadIdx.x, slog = W.stripe_log2;
  uint64_t ext = 0;
  if (lane < W.n_shards) {
    const uint64_t c = W.shards[(uint64_t)lane * kShardStride];
    if (c) ext = ((((c - 1u) >> slog) * (uint64_t)W.n_shards + lane) << slog) + ((c - 1u) & ((1ull << slog) - 1ull)) + 1u;
  }
  for (uint32_t l = 1; l < 64; l <<= 1) {  // (one wave, once per call)
    const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(ext >> 32), (int)l, 64) << 32) |
                       (uint32_t)__shfl_xor((int)(uint32_t)ext, (int)l, 64);
    ext = o > ext ? o : ext;
  }
  if (lane == 0) *W.cursor = ext;
}

// the listed strings as a views subset of the batch (their bytes where they are)
__global__ void k_lean_gather(Batch B, Work W, uint64_t* sub_off, uint32_t* sub_len, uint32_t* sub_tid) {
  const uint32_t count = __hip_atomic_load(W.udefer_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < count; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t idx = W.udefer_list[j];
    const uint64_t so = gld(B.in_off + idx);
    sub_off[j] = so;
    sub_len[j] = B.in_len ? gld(B.in_len + idx) : (uint32_t)min(gld(B.in_off + idx + 1) - so, (uint64_t)0xFFFFFFFFu);
    if (sub_tid) sub_tid[j] = B.table_id ? gld(B.table_id + idx) : 0u;
  }
}

}  // namespace lean

thread_local int lean_stage = 0;  // the step launch_lean failed at (for the host's error message)
int lean_failed_stage() { return lean_stage; }

hipError_t launch_lean(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap, uint64_t* sub_off,
                       uint32_t* sub_len, uint32_t* sub_tid, uint32_t grid_cap, hipStream_t st) {
  lean_stage = 1;
  if (!B.out_len || !B.n || !grid_cap) return hipErrorInvalidValue;
  lean_stage = 2;
  const uint64_t tiles = (B.n + lean::kTile - 1) / lean::kTile;
  const uint32_t grid = (uint32_t)(tiles < grid_cap ? tiles : grid_cap);
  const bool multi = B.table_id != nullptr;
  (void)hipGetLastError();  // (a stale error of an earlier call must not be taken for these launches')
  if (multi) hipLaunchKernelGGL(lean::k_lean<true>, dim3(grid), dim3(lean::kTile), 0, st, B, W, T, out, cap);
  else hipLaunchKernelGGL(lean::k_lean<false>, dim3(grid), dim3(lean::kTile), 0, st, B, W, T, out, cap);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  lean_stage = 3;
  hipLaunchKernelGGL(lean::k_lean_finish, dim3(1), dim3(64), 0, st, W);
  const uint32_t gb = (uint32_t)((B.n + 255) / 256 < 1024 ? (B.n + 255) / 256 : 1024);
  hipLaunchKernelGGL(lean::k_lean_gather, dim3(gb), dim3(256), 0, st, B, W, sub_off, sub_len, multi ? sub_tid : nullptr);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  lean_stage = 4;
  const Batch D{B.bytes, sub_off, B.n, B.out_off, B.status, B.value_id, multi ? sub_tid : nullptr, sub_len, B.out_len,
                W.udefer_list, W.udefer_count};
  return launch_resolve(D, W, T, out, cap, st);
}

hipError_t launch_resolve_deferring(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                                    uint64_t* sub_off, uint32_t* sub_len, uint32_t* sub_tid, hipStream_t st) {
  if (!B.out_len || !B.n) return hipErrorInvalidValue;
  Work W1 = W;
  W1.defer_slow = 1;
  hipError_t e = launch_resolve(B, W1, T, out, cap, st);
  if (e != hipSuccess) return e;
  // the windowed-tile list is the second pass's again
  e = hipMemsetAsync(W.defer_count, 0, sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  const bool multi = B.table_id != nullptr;
  const uint32_t gb = (uint32_t)((B.n + 255) / 256 < 1024 ? (B.n + 255) / 256 : 1024);
  hipLaunchKernelGGL(lean::k_lean_gather, dim3(gb), dim3(256), 0, st, B, W, sub_off, sub_len, multi ? sub_tid : nullptr);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  Work W2 = W;
  W2.defer_slow = 0;
  const Batch D{B.bytes, sub_off, B.n, B.out_off, B.status, B.value_id, multi ? sub_tid : nullptr, sub_len, B.out_len,
                W.udefer_list, W.udefer_count};
  return launch_resolve(D, W2, T, out, cap, st);
}

int lean_blocks_per_cu(int multi) {
  int nb = 0;
  hipError_t e = multi ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lean::k_lean<true>, (int)lean::kTile, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, lean::k_lean<false>, (int)lean::kTile, 0);
  if (e != hipSuccess) (void)hipGetLastError();
  return e == hipSuccess ? nb : 0;
}

}  // namespace ie
