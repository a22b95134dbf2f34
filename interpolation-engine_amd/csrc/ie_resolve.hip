// ie_resolve.hip — k_resolve: interpolate_inserts (py:497-541 / rust-project/src/interp.rs:31-89)
// over a packed batch in ONE pass over HBM.
//
// One 256-lane workgroup per tile of 256 consecutive strings. Packed output: tiles are chained with a
// decoupled look-back over 8-byte {flag, value} words published by agent-scope atomics, and the tile
// index is a ticket each workgroup takes when it starts, so a tile only waits on tiles that have
// started (no assumption about dispatch order). The wait is bounded (10 s): a violation sets the
// exec's error word, which ie_exec_sync / the host APIs report as IE_ERR_TIMEOUT.
// Views output: no look-back, tile = workgroup index. Per tile:
//   1. stage the tile's input bytes in LDS (16-byte loads) and classify every 16-byte chunk into
//      an open-brace and a close-brace mask (plus one "odd byte" bit per chunk: '\' or 0xE3);
//   2. every lane evaluates its string. Clean strings (no odd byte, brace pairs forming chains
//      such as {q-{i}}, keys <= 16 B) take the chain evaluator: pairs are parsed from the masks,
//      then resolved level by level, innermost first, all chains of all lanes of a wave in the
//      same round (one pilot read + one 64-byte entry read per lookup). Everything else takes the
//      exact evaluator (a literal stack evaluation, scratch in global memory), and what that
//      cannot prove equal to the reference goes to the literal path (one wave per string);
//   3. the result of each string is a descriptor (<= 3 top-level pairs and their values) kept
//      in registers; workgroup scan of output lengths, look-back for the tile's global offset;
//   4. lanes copy template runs and value texts into an LDS stage aligned like the destination;
//      the stage streams out with 16-byte stores; offsets, status and value ids are coalesced.
//
// Correctness of the evaluators (DESIGN.md "fast path"): for properly nested strings
// whose spliced values are inert, the reference's rightmost-innermost loop equals a left-to-right
// stack evaluation, and its first failure is the failing pair with the largest opening offset
// (pairs enclosing a failed pair are never evaluated). The chain evaluator only commits strings
// whose every lookup hits an inert value (then any evaluation order gives the reference's bytes);
// any miss or doubt is re-evaluated by the exact evaluator, which reproduces the error order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_device.h"
#include "ie_kernels.h"
#include "ie_literal.h"
#include "ie_bytes.h"

#ifndef IE_WAVES_PER_EU
#define IE_WAVES_PER_EU 4
#endif
// the long-key instances (17-32 byte keys, TF_LONG_KEYS; config 5): their key assembly does not fit
// 128 VGPRs (7 dwords spilled per lane at 4 waves: ~40 MB of scratch writes per config-5 launch)
#ifndef IE_WAVES_PER_EU_LK
#define IE_WAVES_PER_EU_LK 4
#endif

#ifndef IE_RNS
#define IE_RNS r256
#endif

// LEAN5 (an experiment, off: profiles/r06/lean5/README.md): the LEAN first pass in <= 32 KB of LDS
// and <= 96 VGPRs per 256-string tile, i.e. five workgroups (waves) per CU (SIMD) instead of four:
// the chunk masks stay through the chain jobs (a middle level's braces are found from them again, no
// 8 KB of event columns), the job results overwrite their records, one chain job per lane, and the
// output goes to a 13 KB stage, the bytes past it stored straight to HBM by each lane. Measured
// slower than the 4-wave LEAN (config 3 1.38 vs 0.82 ms; the window-loop and two-part variants
// 0.98 / 1.15 ms): every scheme lengthens a tile's life more than the fifth wave adds tiles
#ifndef IE_LEAN5
#define IE_LEAN5 0
#endif
#ifndef IE_WAVES_PER_EU_LEAN
#define IE_WAVES_PER_EU_LEAN 5
#endif

// issue the first value text's loads before the output scan (config 4 first resolve 1.80 -> 1.76 ms,
// configs 2 and 3 unchanged: profiles/r03/early_text/)
#ifndef IE_EARLY_TEXT
#define IE_EARLY_TEXT 1
#endif
#if IE_LEAN5 && !IE_EARLY_TEXT
#error "LEAN5 keeps the entry texts the early loads put in registers (IE_EARLY_TEXT)"
#endif

// chain jobs with wave-uniform skips (empty job slots, no template after the child, short keys):
// config 3 0.856 -> 0.837 ms, VALU -7.4 % per wave (profiles/r04/ab/)
#ifndef IE_JOBS_V2
#define IE_JOBS_V2 1
#endif

// three workgroup barriers fewer per tile (the two scans' trailing barriers, the literal path's when
// no string took it)
#ifndef IE_FEWER_BARRIERS
#define IE_FEWER_BARRIERS 0
#endif

namespace ie {
// everything of one tile size lives in its own namespace: ie_resolve512.hip compiles this file
// again with 512-string tiles (IE_RBLOCK=512, IE_RNS=r512, IE_RESOLVE_WIDE)
namespace IE_RNS {

// value kinds of a descriptor: arena text, literal-path pool result (16-byte units), an entry's
// inline text (entry index; texts <= kInlineText)
enum : uint32_t { kValArena = 1, kValPool = 2, kValEntry = 3 };
constexpr uint32_t kLenMask = (1u << 30) - 1;


// The result of one string: its template with up to kMaxTop top-level pairs [open, close]
// replaced by values. Template run j is [close[j-1] + 1, open[j]) (run 0 starts at 0, the last
// ends at n).
struct Desc {
  uint32_t ntop;
  uint32_t open[kMaxTop], close[kMaxTop];
  uint32_t vk[kMaxTop];  // value kind << 30 | text length
  uint32_t vs[kMaxTop];  // entry index / arena offset / pool offset >> 4
};

__device__ __forceinline__ uint32_t value_kl(uint32_t text_len, uint32_t text_off, uint32_t slot, uint32_t& src) {
  const bool inl = text_len <= kInlineText;
  src = inl ? slot : text_off;
  return ((inl ? kValEntry : kValArena) << 30) | text_len;
}

// the string being evaluated: in the tile's LDS stage (STAGED) or anywhere (a generic pointer:
// flat loads, so one instance serves staged strings and strings past the stage alike)
template <bool STAGED>
struct Src {
  const uint8_t* p;
  __device__ __forceinline__ uint8_t operator[](uint32_t i) const {
    if (STAGED) return ((const lds_u8*)p)[i];
    return p[i];
  }
  __device__ __forceinline__ uint32_t word_at(uintptr_t aligned_addr) const {
    if (STAGED) return *(const lds_u32*)(const lds_u8*)(const uint8_t*)aligned_addr;
    return *(const uint32_t*)aligned_addr;
  }
  __device__ __forceinline__ u32x4 quad_at(uintptr_t aligned16) const {
    if (STAGED) return *(const __attribute__((address_space(3))) u32x4*)(const lds_u8*)(const uint8_t*)aligned16;
    return *(const u32x4*)aligned16;
  }
};

// bytes the skip-ahead scan must look at: '\\' and everything >= 0x7B ('{', '}', U+3020's 0xE3,
// other non-ASCII, '|', '~'). The lowest flagged byte is always a true candidate.
__device__ __forceinline__ uint32_t special_mask(uint32_t w) {
  const uint32_t ge = ((w + 0x05050505u) | w) & 0x80808080u;
  const uint32_t x = w ^ 0x5C5C5C5Cu;
  return ge | ((x - 0x01010101u) & ~x & 0x80808080u);
}

// the top bit of each byte of a special_mask word, as 4 bits
__device__ __forceinline__ uint32_t top_bits(uint32_t m) { return (m * 0x00204081u) >> 28; }

// first index j in [i, n) whose byte is a candidate, else n. Reads aligned 16-byte blocks (one
// never crosses a page, and the LDS stage is padded, so bytes around the string are safe to read
// and ignored): a long template (config 5's 0.4-0.9 KB prompts) is skipped 16 bytes per load.
template <bool STAGED>
__device__ __forceinline__ uint32_t next_special(const Src<STAGED>& s, uint32_t i, uint32_t n) {
  while (i < n) {
    const uintptr_t a = (uintptr_t)(s.p + i);
    const uint32_t sh = (uint32_t)(a & 15);
    const u32x4 q = s.quad_at(a - sh);
    const uint32_t bits = (top_bits(special_mask(q.x)) | (top_bits(special_mask(q.y)) << 4) |
                           (top_bits(special_mask(q.z)) << 8) | (top_bits(special_mask(q.w)) << 12)) &
                          (0xFFFFu << sh);
    if (bits) {
      const uint32_t j = i + (uint32_t)__builtin_ctz(bits) - sh;
      return j < n ? j : n;
    }
    i += 16 - sh;
  }
  return n;
}

// copy len bytes src -> dst: byte head until dst is 4-aligned, dword body with v_alignbyte over
// the source's aligned dwords, byte tail. SRC_LDS / DST_LDS select ds_* vs global access.
template <bool DST_LDS, bool SRC_LDS>
__device__ __forceinline__ void copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src,
                                           uint32_t len) {
  auto rd8 = [&](uint32_t k) -> uint8_t {
    if (SRC_LDS) return ((const lds_u8*)src)[k];
    return gld(src + k);
  };
  auto rd32 = [&](const uint32_t* p, uint32_t q) -> uint32_t {
    if (SRC_LDS) return ((const lds_u32*)(const lds_u8*)(const uint8_t*)p)[q];
    return gld(p + q);
  };
  auto wr8 = [&](uint32_t k, uint8_t v) {
    if (DST_LDS) ((lds_u8*)dst)[k] = v;
    else gst(dst + k, v);
  };
  auto wr32 = [&](uint32_t* p, uint32_t q, uint32_t v) {
    if (DST_LDS) ((lds_u32*)(lds_u8*)(uint8_t*)p)[q] = v;
    else gst(p + q, v);
  };
  uint32_t k = 0;
  while (k < len && (((uintptr_t)(dst + k)) & 3)) {
    wr8(k, rd8(k));
    k++;
  }
  if (k + 4 <= len) {
    const uintptr_t a = (uintptr_t)(src + k);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t* s32 = (const uint32_t*)(a - sh);
    uint32_t* d32 = (uint32_t*)(dst + k);
    const uint32_t nw = (len - k) >> 2;
    // four dwords per step with their loads in flight together (a global source costs one
    // memory round trip per step, not per dword)
    uint32_t q = 0;
    if (sh == 0) {
      for (; q + 4 <= nw; q += 4) {
        const uint32_t a0 = rd32(s32, q), a1 = rd32(s32, q + 1), a2 = rd32(s32, q + 2), a3 = rd32(s32, q + 3);
        wr32(d32, q, a0), wr32(d32, q + 1, a1), wr32(d32, q + 2, a2), wr32(d32, q + 3, a3);
      }
      for (; q < nw; q++) wr32(d32, q, rd32(s32, q));
    } else {
      uint32_t w0 = rd32(s32, 0);
      for (; q + 4 <= nw; q += 4) {
        const uint32_t a1 = rd32(s32, q + 1), a2 = rd32(s32, q + 2), a3 = rd32(s32, q + 3), a4 = rd32(s32, q + 4);
        wr32(d32, q, __builtin_amdgcn_alignbyte(a1, w0, sh));
        wr32(d32, q + 1, __builtin_amdgcn_alignbyte(a2, a1, sh));
        wr32(d32, q + 2, __builtin_amdgcn_alignbyte(a3, a2, sh));
        wr32(d32, q + 3, __builtin_amdgcn_alignbyte(a4, a3, sh));
        w0 = a4;
      }
      for (; q < nw; q++) {
        const uint32_t w1 = rd32(s32, q + 1);
        wr32(d32, q, __builtin_amdgcn_alignbyte(w1, w0, sh));
        w0 = w1;
      }
    }
    k += nw << 2;
  }
  for (; k < len; k++) wr8(k, rd8(k));
}


// ------------------------------------------------------------------------------------------
// Exact evaluator (any string; the reference semantics of SURVEY §3.3). Rounds: every lane scans
// up to its next closing brace, then all lanes that reached one probe the table together.
// Scratch is lane-private LDS: the key buffer (kKeyCap bytes, 4-aligned) and the stack
// (kMaxDepth words, stride kRBlock) reuse the lane's own chain-evaluator columns.
// ------------------------------------------------------------------------------------------
template <bool STAGED>
__device__ uint8_t eval_exact(const DevTable& T, uint32_t tid, const Src<STAGED> s, uint32_t n, bool active, lds_u8* kbuf,
                              lds_u32* stack, Desc& d, uint32_t& out_len, uint32_t& vid, uint32_t& vflags,
                              bool err_keys) {
  constexpr uint8_t kRunning = 0xFF;
  uint8_t status = active ? kRunning : (uint8_t)IE_OK_STR;
  uint32_t depth = 0, klen = 0, vsum = 0, span = 0, ntop = 0;
  uint32_t nopen = 0, nclose = 0;
  bool negclose = false;
  uint32_t poison = 0;  // bit d: the pair open at level d contains a failed pair
  int64_t err_off = -1;
  uint8_t err_cls = 0;
  bool wrapped = false;  // a whole-string pair resolved (typed result so far in wrap_h)
  Hit wrap_h{0, 0, IE_VID_NONE, 0};
  uint32_t i = 0;
  uint32_t c_open = 0, c_ks = 0, c_kl = 0;  // the close waiting for its lookup
  bool c_wrapping = false;

  auto kput = [&](uint8_t c) -> bool {
    if (klen >= (uint32_t)kKeyCap) return false;
    kbuf[klen++] = c;
    return true;
  };
  // end of string: the reference's checks in order (py:516-519, 522, 540)
  auto finish = [&]() -> uint8_t {
    if (nopen == 0) return IE_OK_STR;
    if (nopen != nclose) return IE_E_ASSERT_BRACES;
    if (negclose) return kStatusPending;  // balanced but '}{': py break / rs panic
    // (a key only the host can look up, IE_NEEDS_HOST, or, err_keys, the missing key of an
    // IE_E_INTERP: the literal path reports it with the key)
    if (err_off >= 0) return err_cls == IE_NEEDS_HOST || (err_keys && err_cls == IE_E_INTERP) ? kStatusPending : err_cls;
    if (wrapped) {
      vid = wrap_h.vid;
      vflags = wrap_h.flags;
      return IE_OK_VALUE;
    }
    return IE_OK_STR;
  };

  for (;;) {
    // ---- scan phase: up to this lane's next closing brace ----
    bool need = false;
    while (status == kRunning) {
      if (depth == 0) {
        i = next_special(s, i, n);
      } else {
        const uint32_t j = next_special(s, i, n);
        if (klen + (j - i) > (uint32_t)kKeyCap) {  // long key: literal path
          status = kStatusPending;
          break;
        }
        for (; i < j; i++) kbuf[klen++] = s[i];
      }
      if (i >= n) {
        status = finish();
        break;
      }
      const uint8_t c = s[i];
      if (c == '\\') {
        const uint8_t nx = i + 1 < n ? s[i + 1] : 0;
        if (nx == '{' || nx == '}') {  // an escape pair (py:505-508): plain text
          // '.\}' and '}\}' can restore as '\{...' (py:537-540 replace order): literal path
          if ((nx == '}' && i > 0 && (s[i - 1] == '.' || s[i - 1] == '}')) ||
              (depth && !(kput(c) && kput(nx)))) {
            status = kStatusPending;
            break;
          }
          i += 2;
          continue;
        }
        if (depth && !kput(c)) {
          status = kStatusPending;
          break;
        }
        i++;
        continue;
      }
      if (c == '{') {
        nopen++;
        const uint32_t ks = (klen + 3) & ~3u;  // keys start dword-aligned (pad bytes are not key)
        if (depth >= (uint32_t)kMaxDepth || i >= (1u << 24) || ks > (uint32_t)kKeyCap) {
          status = kStatusPending;
          break;
        }
        stack[depth * kRBlock] = (klen << 24) | i;  // the enclosing key resumes at klen
        klen = ks;
        poison &= ~(1u << depth);
        depth++;
        i++;
        continue;
      }
      if (c == '}') {
        nclose++;
        if (depth == 0) {  // unmatched '}': text, unless the count check fails (py:517-519)
          negclose = true;
          i++;
          continue;
        }
        depth--;
        const uint32_t st = stack[depth * kRBlock];
        const uint32_t open = st & 0xFFFFFFu, resume = st >> 24, ks = (resume + 3) & ~3u;
        c_kl = klen - ks;
        c_ks = ks;
        c_open = open;
        klen = resume;
        if ((poison >> depth) & 1u) {  // an inner pair failed first: never evaluated
          if (depth) poison |= 1u << (depth - 1);
          i++;
          continue;
        }
        // a whole-string pair at this level (get_simple_insertkey truthy, py:510-514)
        c_wrapping = (open == depth) && (i == n - 1 - depth) && (i - open >= 2);
        need = true;
        break;
      }
      if (c == 0xE3 && i + 2 < n && s[i + 1] == 0x80 && s[i + 2] == 0xA0) {
        status = kStatusPending;  // a literal U+3020 collides with the placeholders (py:502-503)
        break;
      }
      if (depth && !kput(c)) {  // other flagged bytes are plain text
        status = kStatusPending;
        break;
      }
      i++;
    }
    if (!__any(need)) break;  // every lane is finished (or pending)
    // ---- lookup phase: all lanes with a pending close probe together ----
    if (need) {
      uint8_t est = 0;
      Hit h;
      int32_t b;
      if (c_wrapping && wrapped) {
        b = find_raw(T, tid, wrap_h, est, h);  // the key is the inner level's raw value
      } else {
        const uint8_t* kg = (const uint8_t*)(kbuf + c_ks);  // generic view of the LDS key
        b = c_kl <= kInlineKey ? find_small(T, tid, (const uint32_t*)kg, c_kl, h) : find_bytes(T, tid, kg, c_kl, h);
        if (b < 0) est = missing_status(T, kg, c_kl);
      }
      if (b >= 0 && !c_wrapping) {
        if (!(h.flags & EF_SPLICE_OK)) {  // py:530 / interp.rs:76-79
          b = -1;
          est = IE_E_ASSERT_TYPE;
        } else if (!(h.flags & EF_INERT)) {
          status = kStatusPending;  // re-resolution / escape hazard
        } else if (depth) {         // splice into the enclosing key
          if (klen + h.text_len > (uint32_t)kKeyCap) {
            status = kStatusPending;
          } else {
            const uint8_t* t = T.arena + h.text_off;
            for (uint32_t k = 0; k < h.text_len; k++) kbuf[klen + k] = gld(t + k);
            klen += h.text_len;
          }
        } else if (ntop == (uint32_t)kMaxTop) {
          status = kStatusPending;  // more top-level pairs than a descriptor holds
        } else {
          uint32_t src;
          const uint32_t kl = value_kl(h.text_len, h.text_off, (uint32_t)b, src);
#pragma unroll
          for (int q = 0; q < kMaxTop; q++) {
            if (ntop == (uint32_t)q) {
              d.open[q] = c_open;
              d.close[q] = i;
              d.vk[q] = kl;
              d.vs[q] = src;
            }
          }
          ntop++;
          vsum += h.text_len;
          span += i - c_open + 1;
        }
      }
      if (b < 0) {
        if ((int64_t)c_open > err_off) {
          err_off = c_open;
          err_cls = est;
        }
        if (depth) poison |= 1u << (depth - 1);
      } else if (c_wrapping) {
        wrapped = true;
        wrap_h = h;
      }
      i++;
    }
  }
  if (active) d.ntop = status == IE_OK_STR ? ntop : 0u;
  out_len = status == IE_OK_STR ? n - span + vsum : 0;
  return status;
}

// ------------------------------------------------------------------------------------------
// Chain evaluator for CLEAN strings (the common case): no '\' or 0xE3 byte, n <= kChainMax, every
// top-level pair a chain (each pair has at most one child: {a}, {q-{i}}, {a-{b-{c-{d}}}}), at most
// kMaxTop chains of depth <= kChainDepth, no whole-string pair, keys <= 16 bytes, every lookup a
// hit on an inert splice-able value. Chains resolve innermost first; round r looks up level r
// (from the bottom) of every chain of every lane at once. A lane that breaks any condition
// returns false with nothing committed; the exact evaluator then decides its result.
// ------------------------------------------------------------------------------------------


struct Probe {
  uint4 q0, q1, q2;
};


// Chain evaluation in two steps. parse_chains (per lane = per string) locates the string's chains
// from the staged event masks; every chain then becomes a JOB, and resolve_jobs runs the jobs of
// the whole tile chain-parallel (a lane per job, two jobs per lane in flight), level by level,
// innermost first; combine_chains (per string) gathers its jobs' results into the descriptor.
// Per-job state is one chain (not a string's three), which keeps the register budget small.
struct ChainJobs {  // LDS views, tile-wide
  lds_u32* crec;    // kJobCap: the chain's record (first open | first close << 8 | innermost open << 16 | last close << 24)
  lds_u16* meta;    // kJobCap: string lane | depth << 12
  lds_u32* res_k;   // kJobCap: the job's result: value kind << 30 | text length; kResFail | status | open << 8; kResReject
  lds_u32* res_s;   // kJobCap: value source (entry index / arena offset)
  lds_u16* p0;      // kRBlock: each string's first byte in the stage
  lds_u32* tbl;     // kRBlock: each string's table in the set
  lds_u64* ev;      // kRBlock x 4 columns: the event masks of strings with chains deeper than 2
  // (LEAN5: no event columns; a middle level's braces come from the classification, kept alive)
  const lds_u32* cm;
  const lds_u32* odd;
  const lds_u32* esc;
  // a small table's pilots staged in LDS (the LEAN instances, T.nb <= kLdsPilots), or null
  const lds_u16* pil;
};
// pilot groups a LEAN workgroup stages in LDS with IE_LDS_PILOTS (tables of up to ~1.4k keys, e.g.
// config 2's 1k-key dict: a lookup is then one memory round trip, the entry's, instead of two); what
// the 4-workgroup LDS budget has left (40,960 B per workgroup). Measured slower (config 2 0.1036 vs
// 0.0994 ms, config 3 0.792 vs 0.774 ms: the second branch costs the kernel 32 B of scratch, and the
// pilots were L2 hits, not the tile's bound), so off by default

constexpr uint32_t kLdsPilots = 352;
constexpr uint32_t kJobCap = kMaxTop * kRBlock;
constexpr uint32_t kResFail = 1u << 29, kResReject = 1u << 28;
constexpr uint32_t kResWhole = 1u << 27;  // a whole-string '{key}' (res_s: the value id; kind bits 0-2)

// The jobs [j0, j0 + 2 * kRBlock) of the tile: lane t takes jobs j0 + t and j0 + kRBlock + t. Round r
// resolves level r of each job (the innermost pair in round 0); the key of a level is A | T | B
// (template before the child, the child's splice text, template after it; a leaf: A only),
// assembled in registers and looked up with one pilot and one 48-byte entry read. A job ends at
// its top level (the value goes to res_k / res_s), at a failure (FAILC: a miss without an
// inserts-dir or an unspliceable hit, recorded with its pair's opening offset) or at anything the
// exact evaluator must decide (kResReject: a long key or text, a non-inert value, a failure when
// !FAILC, a miss an inserts-dir might resolve).
// chain jobs per lane and round: two (their lookups overlap); the long-key instances one: their
// 32-byte key assembly does not fit two jobs in 128 VGPRs (two spilled 7 dwords per lane, 45-76 MB
// of scratch writes per config-5 launch, WRITE_SIZE 1.57-1.95x algorithmic; one job: 1.02x and
// 0.226 -> 0.218 ms, profiles/r05/ab/lk_jobs.txt); at 3 waves per SIMD two jobs fit without a spill
// but run 0.278 ms
#ifndef IE_LK_JOBS
#define IE_LK_JOBS 1
#endif
template <bool LK>
constexpr int kJobsPerLane = LK ? IE_LK_JOBS : 2;
// the LEAN5 instances (96 VGPRs)
#ifndef IE_EXP_NOEVM
#define IE_EXP_NOEVM 0
#endif
#ifndef IE_LEAN_JOBS
#define IE_LEAN_JOBS 1
#endif
template <bool LK, bool L5>
constexpr int kJobsPerLaneOf = L5 ? (LK ? 1 : IE_LEAN_JOBS) : kJobsPerLane<LK>;

template <bool FAILC, bool LK, bool EVM = false>
__device__ void resolve_jobs(const DevTable& T, const lds_u8* tile, const ChainJobs J, uint32_t j0, uint32_t njobs,
                             bool& chain_fail, uint64_t* stamp) {
  constexpr int NJ = kJobsPerLaneOf<LK, EVM>;
  const uint32_t tid = threadIdx.x;
  bool on[NJ], done[NJ], wh[NJ];
  uint32_t job[NJ], cr[NJ], dep[NJ], ls[NJ], tb[NJ], res_k[NJ], res_s[NJ];
  const lds_u8* s[NJ];
  uint32_t ct[NJ][4], ctl[NJ], co_[NJ], cl_[NJ];
  uint32_t maxd = 0;
#pragma unroll
  for (int q = 0; q < NJ; q++) {
    job[q] = j0 + (uint32_t)q * kRBlock + tid;
    const bool valid = job[q] < njobs;
    cr[q] = valid ? J.crec[job[q]] : 0u;
    const uint32_t mt = valid ? (uint32_t)J.meta[job[q]] : 0u;
    ls[q] = mt & 0xFFFu;
    dep[q] = valid ? (mt >> 12) & 7u : 0u;
    wh[q] = valid && (mt >> 15) != 0u;  // a whole-string '{key}': the raw value, any type
    s[q] = tile + (valid ? (uint32_t)J.p0[ls[q]] : 0u);
    tb[q] = valid ? J.tbl[ls[q]] : 0u;
    done[q] = !valid;
    res_k[q] = kResReject;
    res_s[q] = 0;
    ct[q][0] = ct[q][1] = ct[q][2] = ct[q][3] = 0;
    ctl[q] = co_[q] = cl_[q] = 0;
    maxd = dep[q] > maxd ? dep[q] : maxd;
  }
  const uint32_t R = w_max32(maxd);
  for (uint32_t r = 0; r < R; r++) {
    uint32_t open[NJ], close[NJ], la[NJ], lb[NJ], klen[NJ], slot[NJ];
    u32x4 ka[NJ], kb[NJ], kw[NJ];
    uint64_t h[NJ];
    u32x4 kw2[NJ];  // bytes 16..31 of an innermost key longer than the entry's inline copy
    bool lk[NJ];
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      on[q] = !done[q] && r < dep[q];
      // level r: the innermost pair in round 0, the outermost in the last round; a middle level is
      // the open before the previous level's and the close after it (from the string's masks)
      const bool top = r + 1 == dep[q];
      uint32_t o = r == 0 ? cr_inner_open(cr[q]) : top ? cr_first_open(cr[q]) : 0u;
      uint32_t c = r == 0 ? cr_first_close(cr[q]) : top ? cr_last_close(cr[q]) : 0u;
      const bool mid = on[q] && r != 0 && !top;
      if (__any(mid)) {
        if (EVM && !IE_EXP_NOEVM) {
          // the string's events again, from the tile's chunk masks (up to the chain's last close:
          // every level of the chain lies before it)
          bool evok = mid, evesc;
          Ev Om, Cm;
          string_events(tile, (uint32_t)(s[q] - tile), cr_last_close(cr[q]) + 1u, J.cm, J.odd, J.esc, evok, evesc, Om, Cm);
          if (mid) {
            o = ev_last(ev_below(Om, co_[q]));
            c = ev_first(ev_from(Cm, cl_[q] + 1u));
          }
        } else if (mid) {
          const lds_u64* e = J.ev + ls[q];
          o = ev_last(ev_below(Ev{e[0], e[kRBlock]}, co_[q]));
          c = ev_first(ev_from(Ev{e[2 * kRBlock], e[3 * kRBlock]}, cl_[q] + 1u));
        }
      }
      open[q] = on[q] ? o : 0u;
      close[q] = on[q] ? c : 0u;
      la[q] = on[q] ? (r == 0 ? close[q] : co_[q]) - open[q] - 1 : 0u;
      lb[q] = on[q] && r != 0 ? close[q] - cl_[q] - 1 : 0u;
#if IE_JOBS_V2
      // (uniform skips: a slot no lane of the wave uses, the template after the child when no lane
      // has one, e.g. config 3's {q-{iM}})
      ka[q] = kb[q] = u32x4{0, 0, 0, 0};
      if (__any(on[q])) ka[q] = ld16a(s[q] + open[q] + 1);
      if (r != 0 && __any(lb[q] != 0u)) kb[q] = ld16a(s[q] + cl_[q] + 1);
#else
      ka[q] = ld16a(s[q] + open[q] + 1);
      kb[q] = r != 0 ? ld16a(s[q] + cl_[q] + 1) : u32x4{0, 0, 0, 0};
#endif
    }
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      klen[q] = la[q] + (r != 0 ? ctl[q] + lb[q] : 0u);
      // LK (a table with 17-32 byte keys): an innermost key (template bytes only) that long has
      // its tail compared with the arena's copy of the entry's key once the entry is in
      lk[q] = LK && on[q] && r == 0 && klen[q] > 16u && klen[q] <= 32u;
      kw2[q] = lk[q] ? keep_bytes(ld16a(s[q] + open[q] + 17), klen[q] - 16u) : u32x4{0, 0, 0, 0};
      if (on[q] && klen[q] > 16u && !lk[q]) {  // longer keys live in the arena: exact evaluator
        on[q] = false;
        done[q] = true;
      }
#if IE_JOBS_V2
      h[q] = 0;
      kw[q] = u32x4{0, 0, 0, 0};
      if (!__any(on[q])) continue;
      // the parts are exact (template bytes masked, the child's text zero past its length, shifts
      // drop what passes 16 bytes): no final mask
      u32x4 k = keep_bytes(ka[q], la[q]);
      if (r != 0) {
        const u32x4 t = shl_bytes(u32x4{ct[q][0], ct[q][1], ct[q][2], ct[q][3]}, la[q]);
        k = u32x4{k.x | t.x, k.y | t.y, k.z | t.z, k.w | t.w};
        if (__any(lb[q] != 0u)) {
          const u32x4 b = shl_bytes(keep_bytes(kb[q], lb[q]), la[q] + ctl[q]);
          k = u32x4{k.x | b.x, k.y | b.y, k.z | b.z, k.w | b.w};
        }
      }
      kw[q] = k;
      uint64_t hh = hash_init(klen[q], T.seed, tb[q]);
      if (klen[q] > 0u) hh = hash_word(hh, kw[q].x);
      if (klen[q] > 4u) hh = hash_word(hh, kw[q].y);
      if (__any(klen[q] > 8u)) {
        if (klen[q] > 8u) hh = hash_word(hh, kw[q].z);
        if (klen[q] > 12u) hh = hash_word(hh, kw[q].w);
      }
#else
      u32x4 k = keep_bytes(ka[q], la[q]);
      if (r != 0) {
        const u32x4 t = shl_bytes(u32x4{ct[q][0], ct[q][1], ct[q][2], ct[q][3]}, la[q]);
        const u32x4 b = shl_bytes(keep_bytes(kb[q], lb[q]), la[q] + ctl[q]);
        k = u32x4{k.x | t.x | b.x, k.y | t.y | b.y, k.z | t.z | b.z, k.w | t.w | b.w};
      }
      kw[q] = keep_bytes(k, klen[q]);
      uint64_t hh = hash_init(klen[q], T.seed, tb[q]);
      if (klen[q] > 0u) hh = hash_word(hh, kw[q].x);
      if (klen[q] > 4u) hh = hash_word(hh, kw[q].y);
      if (klen[q] > 8u) hh = hash_word(hh, kw[q].z);
      if (klen[q] > 12u) hh = hash_word(hh, kw[q].w);
#endif
      if (LK && klen[q] > 16u) hh = hash_word(hh, kw2[q].x);
      if (LK && klen[q] > 20u) hh = hash_word(hh, kw2[q].y);
      if (LK && klen[q] > 24u) hh = hash_word(hh, kw2[q].z);
      if (LK && klen[q] > 28u) hh = hash_word(hh, kw2[q].w);
      h[q] = hh;
    }
    if (stamp && threadIdx.x == 0 && r == 0) {  // diagnostic: keys hashed
      asm volatile("" ::"v"(h[0]), "v"(h[1]));
      stamp[6] = __builtin_amdgcn_s_memrealtime();
    }
#ifdef IE_CUCKOO
    // two-choice table: both candidate entries in one round (one memory latency per level)
    uint32_t slot2[NJ];
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      uint32_t a = 0, b = 0;
      if (on[q]) ck_slots(h[q], T.m, a, b);
      slot[q] = a;
      slot2[q] = b;
    }
#else
    // pilots, then entries: two memory latencies per round, every job's in flight together (a
    // small table's pilots: from LDS, one memory latency per round)
    if (J.pil) {
#pragma unroll
      for (int q = 0; q < NJ; q++) {
        const uint32_t pilot = on[q] ? (uint32_t)J.pil[ph_group(h[q], T.nb)] : 0u;
        slot[q] = on[q] ? ph_slot(h[q], pilot, T.m) : 0u;
      }
    } else {
#pragma unroll
      for (int q = 0; q < NJ; q++) {
        const uint32_t pilot = on[q] ? (uint32_t)gld(T.pilots + ph_group(h[q], T.nb)) : 0u;
        slot[q] = on[q] ? ph_slot(h[q], pilot, T.m) : 0u;
      }
    }
#endif
    if (stamp && threadIdx.x == 0 && r == 0) {  // diagnostic: pilots arrived
      asm volatile("" ::"v"(slot[0]), "v"(slot[1]));
      stamp[13] = __builtin_amdgcn_s_memrealtime();
    }
    Probe P[NJ];
    uint32_t wvid[NJ];
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      wvid[q] = IE_VID_NONE;
      if (__any(on[q])) {
        const uint4* e = (const uint4*)(T.entries + slot[q]);
        P[q].q0 = gld4(e);
        P[q].q1 = gld4(e + 1);
        P[q].q2 = gld4(e + 2);
#ifdef IE_CUCKOO
        const uint4* e2 = (const uint4*)(T.entries + slot2[q]);
        const uint4 b0 = gld4(e2), b1 = gld4(e2 + 1), b2 = gld4(e2 + 2);
        // the second candidate holds the key: take it (its slot, its words)
        const bool sb = on[q] && entry_head_ok(b0, klen[q], tb[q]) & (b1.x == kw[q].x) & (b1.y == kw[q].y) &
                        (b1.z == kw[q].z) & (b1.w == kw[q].w);
        if (sb) {
          P[q].q0 = b0, P[q].q1 = b1, P[q].q2 = b2;
          slot[q] = slot2[q];
        }
#endif
        if (__any(on[q] && wh[q])) wvid[q] = on[q] && wh[q] ? gld(&T.entries[slot[q]].vid) : IE_VID_NONE;
      }
    }
    if (stamp && threadIdx.x == 0 && r < 2) {  // diagnostic: entries arrived
      asm volatile("" ::"v"(P[0].q0.x), "v"(P[1].q0.x), "v"(P[0].q2.x));
      stamp[14 + r] = __builtin_amdgcn_s_memrealtime();
    }
#pragma unroll
    for (int q = 0; q < NJ; q++) {
      if (!__any(on[q])) continue;
      const Probe& E = P[q];
      bool hit = on[q] && (entry_head_ok(E.q0, klen[q], tb[q]) & (E.q1.x == kw[q].x) & (E.q1.y == kw[q].y) &
                           (E.q1.z == kw[q].z) & (E.q1.w == kw[q].w));
      if (LK && __any(lk[q] && hit)) {  // the tail of a long key: the arena's copy (key_off_of), bytes 16..
        u32x4 tail{0, 0, 0, 0};
        if (lk[q] && hit) {
          const uint32_t* kp = (const uint32_t*)(T.arena + key_off_of(E.q0.w, E.q0.y) + 16u);
          tail = keep_bytes(u32x4{gld(kp), gld(kp + 1), gld(kp + 2), gld(kp + 3)}, klen[q] - 16u);
        }
        hit = hit && (!lk[q] || ((tail.x == kw2[q].x) & (tail.y == kw2[q].y) & (tail.z == kw2[q].z) & (tail.w == kw2[q].w)));
      }
      const uint32_t flags = E.q0.z, tlen = E.q0.y;
      // (a whole-string '{key}' takes any hit: its result is the raw value, nothing is spliced)
      const bool good = hit && (wh[q] || ((flags & EF_SPLICE_OK) && (flags & EF_INERT)));
      // a miss (no inserts-dir: py:465 / interp.rs:136) or a hit that cannot be spliced
      // (py:530 / interp.rs:76-79) fails this pair; a hit on a value needing care, or a miss that
      // the inserts-dir might resolve, goes to the exact evaluator
      const bool would_fail =
          on[q] && ((!hit && !(T.flags & TF_HAS_DIR)) || (hit && !wh[q] && !(flags & EF_SPLICE_OK)));
      chain_fail |= would_fail;  // the adaptive variant choice counts these (either variant)
      const bool fail = FAILC && would_fail;
      const bool top = r + 1 == dep[q];
      if (on[q] && !good && !fail) done[q] = true;  // kResReject
      if (fail) {
        res_k[q] = kResFail | (hit ? (uint32_t)IE_E_ASSERT_TYPE : (uint32_t)IE_E_INTERP) | (open[q] << 8);
        done[q] = true;
      }
      if (on[q] && good && !top) {  // inner level: this text goes into the parent's key
        if (tlen > 16u) done[q] = true;  // kResReject
        ct[q][0] = E.q2.x, ct[q][1] = E.q2.y, ct[q][2] = E.q2.z, ct[q][3] = E.q2.w;
        ctl[q] = tlen;
        co_[q] = open[q];
        cl_[q] = close[q];
      }
      if (on[q] && good && top) {
        uint32_t src;
        res_k[q] = wh[q] ? (kResWhole | (flags & EF_KIND_MASK)) : value_kl(tlen, E.q0.w, slot[q], src);
        res_s[q] = wh[q] ? wvid[q] : src;
        done[q] = true;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NJ; q++) {
    if (job[q] < njobs) {
      J.res_k[job[q]] = res_k[q];
      J.res_s[job[q]] = res_s[q];
    }
  }
}

// a string's descriptor from its jobs [jb, jb + nch): false when any job needs the exact evaluator;
// a failed job (FAILC) makes the string fail with the status of the failing pair with the largest
// opening offset (the reference resolves the rightmost chain first and stops at its first failure)
// (RECS_LDS: the chain records are read from the job array, not kept in registers across the jobs;
// the LEAN5 layout overwrites them with the results, so it passes them in registers)
template <bool RECS_LDS>
__device__ bool combine_chains(const ChainJobs J, uint32_t jb, uint32_t nch, const uint32_t (&crec)[kMaxTop],
                               uint32_t n, Desc& d, uint32_t& out_len, uint8_t& status, uint32_t& vid,
                               uint32_t& vflags) {
  if (nch == 1u) {  // a whole-string '{key}' job: its raw value is the typed result (py:510-514)
    const uint32_t rk = J.res_k[jb];
    if ((rk & kResWhole) && !(rk & (kResFail | kResReject)) && (rk >> 30) == 0u) {
      d.ntop = 0;
      out_len = 0;
      status = IE_OK_VALUE;
      vid = J.res_s[jb];
      vflags = rk & EF_KIND_MASK;
      return true;
    }
  }
  bool ok = true;
  uint32_t fw = 0, vsum = 0, span = 0;
#pragma unroll
  for (int c = 0; c < kMaxTop; c++) {
    if ((uint32_t)c >= nch) continue;
    const uint32_t rk = J.res_k[jb + c], rs = J.res_s[jb + c];
    const uint32_t rec = RECS_LDS ? J.crec[jb + c] : crec[c];
    const uint32_t a = cr_first_open(rec), e = cr_last_close(rec);
    if (rk & kResReject) {
      ok = false;
    } else if ((rk >> 30) == 0u) {  // failed at the pair opening at (rk >> 8) & 0xFF
      const uint32_t op = (rk >> 8) & 0x3FFFu;  // (14 bits: the flat pairs of long strings)
      if ((fw & 0xFFu) == 0u || op > (fw >> 8)) fw = (op << 8) | (rk & 0xFFu);
    } else {
      d.open[c] = a;
      d.close[c] = e;
      d.vk[c] = rk;
      d.vs[c] = rs;
      vsum += rk & kLenMask;
      span += e - a + 1;
    }
  }
  const bool failed = (fw & 0xFFu) != 0u;
  d.ntop = ok && !failed ? nch : 0u;
  out_len = ok && !failed ? n - span + vsum : 0u;
  if (ok && failed) status = (uint8_t)(fw & 0xFFu);
  return ok;
}

// ------------------------------------------------------------------------------------------
// decoupled look-back (wave 0 of the workgroup, all 64 lanes). Words: flag<<62 | value.
// ------------------------------------------------------------------------------------------
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagIncl = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ void publish(uint64_t* state, uint32_t tile, uint64_t word) {
  __hip_atomic_store(state + tile, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the tile's aggregate (or, for tile 0, its inclusive prefix) as soon as it is known
__device__ __forceinline__ void publish_aggregate(uint64_t* state, uint32_t tile, uint64_t agg) {
  if (lane_id() == 0) publish(state, tile, (tile == 0 ? kFlagIncl : kFlagAgg) | agg);
}

// one poll: the words of the 64 predecessors pos, pos-1, ..., pos-63 (lane l at distance l)
__device__ __forceinline__ uint64_t lb_poll(const uint64_t* state, int64_t pos) {
  const int64_t idx = pos - (int64_t)lane_id();
  return idx >= 0 ? __hip_atomic_load(state + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagIncl;
}

// the exclusive prefix of `tile` from its predecessors' words; publishes the inclusive prefix.
// `early` is a first poll issued before the output build (its latency hides behind the build);
// if it shows a gap the window is simply polled again.
__device__ uint64_t look_back(uint64_t* state, uint32_t tile, uint64_t agg, uint32_t* err,
                              uint32_t* polls, uint64_t early) {
  const uint32_t lane = lane_id();
  if (tile == 0) return 0;
  uint64_t excl = 0;
  int64_t pos = (int64_t)tile - 1;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t nap = 1, npoll = 0;
  // each poll reads a window of 64 predecessors (lane l at distance l from pos): one 512-byte
  // request; a window with a gap before its first inclusive word is re-read after a backoff
  for (bool use_early = true;; use_early = false) {
    const uint64_t w = use_early ? early : lb_poll(state, pos);
    const uint64_t flag = w >> 62;
    const uint64_t incl_m = __ballot(flag == 2);
    const uint64_t wait_m = __ballot(flag == 0);
    const uint32_t first = incl_m ? (uint32_t)__builtin_ctzll(incl_m) : 64u;
    const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
    if (wait_m & need) {
      if (use_early) continue;  // the early poll was too early: poll now, no backoff
      npoll++;
      // backoff: 64 * nap cycles, doubling up to ~1 us
      for (uint32_t k = 0; k < nap; k++) __builtin_amdgcn_s_sleep(1);
      nap = nap < 32 ? 2 * nap : 32;
      // bounded spin: 10 s of s_memrealtime (100 MHz); a missing predecessor is a bug
      if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      continue;
    }
    excl += w_sum(lane <= first ? (w & kValMask) : 0ull);
    if (first < 64) break;
    pos -= 64;
  }
  if (lane == 0) publish(state, tile, kFlagIncl | (excl + agg));
  if (polls && lane == 0 && npoll) atomicAdd(polls, npoll);  // telemetry (diagnostic runs only)
  return excl;
}

// ------------------------------------------------------------------------------------------
// workgroup scan helper
// ------------------------------------------------------------------------------------------
// TRAIL: a second barrier so that lds_w can be written again at once; without it the caller
// guarantees a barrier before the next write of lds_w
template <bool TRAIL = true>
__device__ uint64_t block_scan(uint64_t v, uint64_t* lds_w, uint64_t* total) {
  const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) lds_w[wid] = inc;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kRBlock / 64; w++) {
    const uint64_t x = lds_w[w];
    if (w < wid) base += x;
    tot += x;
  }
  if (TRAIL) __syncthreads();
  *total = tot;
  return base + inc - v;
}

// Union region, by phase:
//   classification + evaluation: key areas [0, kKbufLds) | exact-evaluator stacks
//     [kKbufLds, kEvalLds) | chunk event masks [kCmOff, ..) | odd-chunk bits [kOddOff, ..)
//     (the masks are read only while building a lane's event window)
//   literal results: pool offsets at [0, 4 * kRBlock)
//   output: the tile's output bytes (tile-relative), read back for the realigned stream-out
constexpr uint32_t kKbufLds = kRBlock * kKeyCap;
constexpr uint32_t kStackLds = kRBlock * 32;  // exact-evaluator stacks (kMaxDepth words) | chain event masks
constexpr uint32_t kEvalLds = kKbufLds + kStackLds;
constexpr uint32_t kChunks = (kRTileBytes + 32) / 16;
constexpr uint32_t kOddWords = ((kChunks + kRBlock - 1) / kRBlock) * (kRBlock / 32) + 2;
constexpr uint32_t kCmOff = kEvalLds;
constexpr uint32_t kOddOff = kCmOff + 4 * (kChunks + 10);
constexpr uint32_t kEscOff = kOddOff + 4 * kOddWords;
constexpr uint32_t kClassEnd = kEscOff + 4 * kOddWords;
constexpr uint32_t kUnionLds = kClassEnd > (uint32_t)kRStageBytes + 32 ? kClassEnd : (uint32_t)kRStageBytes + 32;
// the output stage: all of the union the classification needs anyway (config 2's 256-string
// tiles average 20.4 KB of output; a 20 KB stage sent a third of them to k_emit_windows)
constexpr uint32_t kOutStage = (kUnionLds - 32) & ~15u;
static_assert(4 * kRBlock + 13 * 4 * kRBlock <= kUnionLds, "parked descriptors fit the union");
static_assert(kKeyCap >= 32 && kMaxDepth <= 8, "evaluator scratch");

// LEAN5 union, by phase: classification (chunk masks, odd / escape bits) from the staging through the
// chain jobs | the job arrays (records, overwritten by their results; meta; result sources; string
// starts); then the output's first kLWin bytes over all of it (the rest over the input stage)
constexpr uint32_t kLCmOff = 0;
constexpr uint32_t kLOddOff = kLCmOff + 4 * (kChunks + 10);
constexpr uint32_t kLEscOff = kLOddOff + 4 * kOddWords;
constexpr uint32_t kLCrecOff = (kLEscOff + 4 * kOddWords + 15) & ~15u;
constexpr uint32_t kLMetaOff = kLCrecOff + 4 * kJobCap;
constexpr uint32_t kLResSOff = kLMetaOff + 2 * kJobCap;
constexpr uint32_t kLP0Off = kLResSOff + 4 * kJobCap;
constexpr uint32_t kUnionLean = (kLP0Off + 2 * kRBlock + 15) & ~15u;
constexpr uint32_t kLWin = kUnionLean - 16;  // the output window (a multiple of 16; the unaligned
                                             // stream-out reads one block past it)
// the most output a LEAN5 tile writes itself (the window, then straight stores); more: k_emit_windows
constexpr uint32_t kLDirectMax = 2 * kLWin;

// where a tile's strings lie: [lo, hi) for the tile, this lane's string at so (sn bytes)
struct TileGeo {
  uint64_t lo, hi, so, sn;
};
__device__ __forceinline__ TileGeo load_geo(const Batch& B, uint32_t tile, uint32_t tid) {
  TileGeo g{0, 0, 0, 0};
  const uint64_t first = (uint64_t)tile * kRBlock;
  if (first >= B.n) return g;
  const uint64_t last = min(first + (uint64_t)kRBlock, B.n), i = first + tid;
  g.lo = gld(B.in_off + first);
  if (B.in_len) {  // views input: the tile's span ends with its last string (nothing staged if it
                   // lies before the first: such strings are read where they are)
    const uint64_t e = gld(B.in_off + last - 1) + gld(B.in_len + last - 1);
    g.hi = e > g.lo ? e : g.lo;
  } else {
    g.hi = gld(B.in_off + last);
  }
  if (i < B.n) {
    g.so = gld(B.in_off + i);
    g.sn = B.in_len ? (uint64_t)gld(B.in_len + i) : gld(B.in_off + i + 1) - g.so;
  }
  return g;
}

// byte length of input string i (packed or views input)
__device__ __forceinline__ uint64_t in_length(const Batch& B, uint64_t i) {
  return B.in_len ? (uint64_t)gld(B.in_len + i) : gld(B.in_off + i + 1) - gld(B.in_off + i);
}

constexpr uint32_t kStageChunks = (kRTileBytes + 31) / 16;  // the input stage: the tile's first chunks

// a tile's input chunks in flight into registers, written to the LDS stage later
template <int MAXV>
struct TilePrefetch {
  uint4 v[MAXV];
  uint32_t nv;
  __device__ __forceinline__ void issue(const Batch& B, const TileGeo& g, uint32_t tid) {
    const uintptr_t plo = (uintptr_t)(B.bytes + g.lo);
    const uint32_t shift = (uint32_t)(plo & 15);
    const uint4* src = (const uint4*)(plo - shift);  // an aligned chunk never crosses a page
    nv = (uint32_t)min((uint64_t)((shift + (g.hi - g.lo) + 15) >> 4), (uint64_t)kStageChunks);
#pragma unroll
    for (int k = 0; k < MAXV; k++) {
      const uint32_t j = tid + (uint32_t)k * kRBlock;
      if (j < nv) v[k] = gld4s(src + j);
    }
  }
  __device__ __forceinline__ void commit(uint4* dst, uint32_t tid) const {
#pragma unroll
    for (int k = 0; k < MAXV; k++) {
      const uint32_t j = tid + (uint32_t)k * kRBlock;
      if (j < nv) dst[j] = v[k];
    }
  }
};
constexpr int kStageV = (kStageChunks + kRBlock - 1) / kRBlock;

// bytes r..r+15 (r wave-uniform, 0..15) of the 32 bytes x | y
__device__ __forceinline__ uint4 bytes_at(u32x4 x, u32x4 y, uint32_t r) {
  const uint32_t sb = r & 3u;
  uint32_t a0, a1, a2, a3, a4;
  switch (r >> 2) {  // uniform
    case 0: a0 = x.x, a1 = x.y, a2 = x.z, a3 = x.w, a4 = y.x; break;
    case 1: a0 = x.y, a1 = x.z, a2 = x.w, a3 = y.x, a4 = y.y; break;
    case 2: a0 = x.z, a1 = x.w, a2 = y.x, a3 = y.y, a4 = y.z; break;
    default: a0 = x.w, a1 = y.x, a2 = y.y, a3 = y.z, a4 = y.w; break;
  }
  return make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sb), __builtin_amdgcn_alignbyte(a2, a1, sb),
                    __builtin_amdgcn_alignbyte(a3, a2, sb), __builtin_amdgcn_alignbyte(a4, a3, sb));
}

// stream the LDS stage [0, len) to g (any alignment): 16-byte stores at 16-byte aligned
// addresses, each assembled from the two stage blocks it straddles; byte stores at the ends
// (STAGE: the stage's capacity, which bounds the blocks per lane)
template <uint32_t STAGE = kOutStage>
__device__ __forceinline__ void stream_stage(uint8_t* g, const uint8_t* stage, uint32_t len, uint32_t tid) {
  const uintptr_t pg = (uintptr_t)g, pe = pg + len;
  const uintptr_t a_up = (pg + 15) & ~(uintptr_t)15, b_down = pe & ~(uintptr_t)15;
  if (a_up >= b_down) {
    for (uint32_t k = tid; k < len; k += kRBlock) gst(g + k, ((const lds_u8*)stage)[k]);
    return;
  }
  const uint32_t head = (uint32_t)(a_up - pg), tail = (uint32_t)(pe - b_down);
  if (tid < head) gst(g + tid, ((const lds_u8*)stage)[tid]);
  if (tid < tail) {
    const uint32_t k = (uint32_t)(b_down - pg) + tid;
    gst(g + k, ((const lds_u8*)stage)[k]);
  }
  const uint32_t nv = (uint32_t)((b_down - a_up) >> 4);
  constexpr int kOutV = (STAGE + kRBlock * 16 - 1) / (kRBlock * 16);
  uint4 v[kOutV];
  if (head == 0) {  // (uniform) a 16-aligned destination, e.g. reserved ranges: the stage's blocks as they are
#pragma unroll
    for (int k = 0; k < kOutV; k++) {
      const uint32_t c = tid + (uint32_t)k * kRBlock;
      if (c < nv) {
        const u32x4 x = ((const lds_u128*)(const lds_u8*)stage)[c];
        v[k] = make_uint4(x.x, x.y, x.z, x.w);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kOutV; k++) {
      const uint32_t c = tid + (uint32_t)k * kRBlock;
      if (c < nv) {
        const lds_u128* blk = (const lds_u128*)(const lds_u8*)stage + c;
        const u32x4 x = blk[0], y = blk[1];
        v[k] = bytes_at(x, y, head);
      }
    }
  }
  uint4* dstv = (uint4*)a_up;
#pragma unroll
  for (int k = 0; k < kOutV; k++) {
    const uint32_t c = tid + (uint32_t)k * kRBlock;
    if (c < nv) gst4s(dstv + c, v[k]);
  }
}

// the whole wave copies len bytes src -> dst (LDS; arguments uniform): lane k moves destination
// dwords k, k+64, ... realigned from the source's aligned dwords (reads at most 3 bytes past the
// source end, inside an aligned dword)
template <bool SRC_LDS>
__device__ void wave_copy(lds_u8* dst, const uint8_t* src, uint32_t len) {
  auto rd8 = [&](const uint8_t* p) -> uint8_t {
    if (SRC_LDS) return *(const lds_u8*)p;
    return gld(p);
  };
  auto rd32 = [&](const uint32_t* p) -> uint32_t {
    if (SRC_LDS) return *(const lds_u32*)(const lds_u8*)(const uint8_t*)p;
    return gld(p);
  };
  const uint32_t lane = lane_id();
  const uint32_t h0 = (0u - (uint32_t)(uintptr_t)dst) & 3u, h = h0 < len ? h0 : len;
  if (lane < h) dst[lane] = rd8(src + lane);
  const uint32_t nw = (len - h) >> 2;
  const uintptr_t sa = (uintptr_t)(src + h);
  const uint32_t sh = (uint32_t)(sa & 3u);
  const uint32_t* s32 = (const uint32_t*)(sa - sh);
  lds_u32* d32 = (lds_u32*)(dst + h);
  uint32_t q = lane;
  for (; q + 192 < nw; q += 256) {  // 1 KB per step, every load of the step in flight together
    uint32_t a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = rd32(s32 + q + 64 * k), b[k] = rd32(s32 + q + 64 * k + 1);
#pragma unroll
    for (int k = 0; k < 4; k++) d32[q + 64 * k] = sh ? __builtin_amdgcn_alignbyte(b[k], a[k], sh) : a[k];
  }
  for (; q < nw; q += 64) {
    const uint32_t w0 = rd32(s32 + q);
    d32[q] = sh ? __builtin_amdgcn_alignbyte(rd32(s32 + q + 1), w0, sh) : w0;
  }
  const uint32_t t0 = h + 4 * nw;
  if (lane < len - t0) dst[t0 + lane] = rd8(src + t0 + lane);
}

// the part of one output piece (len bytes at src, first byte at window position rel) inside the
// window [0, wl): short parts by their own lane, long ones by the whole wave
template <bool SRC_LDS>
__device__ __forceinline__ void window_piece(lds_u8* win, int64_t rel, const uint8_t* src, uint32_t len, uint32_t wl) {
  const int64_t a = rel > 0 ? rel : 0, b = rel + (int64_t)len < (int64_t)wl ? rel + (int64_t)len : (int64_t)wl;
  const uint32_t n = a < b ? (uint32_t)(b - a) : 0u;
  const uint8_t* from = src + (a - rel);
  const bool big = n > 96u;
  if (n && !big) copy_bytes<true, SRC_LDS>((uint8_t*)(win + a), from, n);
  for (uint64_t m = __ballot(big); m; m &= m - 1) {
    const int l = __builtin_ctzll(m);
    const uint64_t f = (uint64_t)(uintptr_t)from;
    const uint32_t fl = __shfl((uint32_t)f, l, 64), fh = __shfl((uint32_t)(f >> 32), l, 64);
    const uint32_t aa = __shfl((uint32_t)a, l, 64), nn = __shfl(n, l, 64);
    wave_copy<SRC_LDS>(win + aa, (const uint8_t*)(uintptr_t)(((uint64_t)fh << 32) | fl), nn);
  }
}

// len (<= 28) bytes held as 8 little-endian words (zero past the text) to any global address: head
// bytes until 4-aligned, then dwords realigned in registers, then the tail bytes (put_words' twin)
__device__ __forceinline__ void put_words_g(uint8_t* dst, const uint32_t (&t)[8], uint32_t len) {
  const uint32_t h0 = (0u - (uint32_t)(uintptr_t)dst) & 3u, h = h0 < len ? h0 : len;
  if (h > 0) gst(dst, (uint8_t)t[0]);
  if (h > 1) gst(dst + 1, (uint8_t)(t[0] >> 8));
  if (h > 2) gst(dst + 2, (uint8_t)(t[0] >> 16));
  const uint32_t rest = len - h, nfull = rest >> 2, r = rest & 3u;
  uint32_t* q = (uint32_t*)(dst + h);
  uint32_t last = 0;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const uint32_t a = __builtin_amdgcn_alignbyte(t[k + 1], t[k], h);  // text bytes h+4k .. h+4k+3
    if ((uint32_t)k < nfull) gst(q + k, a);
    last = (uint32_t)k == nfull ? a : last;
  }
  uint8_t* b = dst + h + 4u * nfull;
  for (uint32_t k = 0; k < r; k++) gst(b + k, (uint8_t)(last >> (8u * k)));
}

// len bytes at src (global memory) -> stage + off, by this lane; pieces over 96 bytes (multi-KB
// values such as a state's history) by the whole wave instead, so that one lane's long copy does
// not hold up its tile (and with it every later tile's look-back). Uniform control flow.
__device__ __forceinline__ void stage_piece(lds_u8* stage, bool on, uint32_t off, const uint8_t* src, uint32_t len) {
  const bool big = on && len > 96u;
  if (on && !big && len) copy_bytes<true, false>((uint8_t*)(stage + off), src, len);
  for (uint64_t m = __ballot(big); m; m &= m - 1) {
    const int l = __builtin_ctzll(m);
    const uint64_t f = (uint64_t)(uintptr_t)src;
    const uint32_t fl = __shfl((uint32_t)f, l, 64), fh = __shfl((uint32_t)(f >> 32), l, 64);
    const uint32_t oo = __shfl(off, l, 64), nn = __shfl(len, l, 64);
    wave_copy<false>(stage + oo, (const uint8_t*)(uintptr_t)(((uint64_t)fh << 32) | fl), nn);
  }
}

// The unescape command's recursive_interpolate (py:1463-1464): an item that is a whole-string
// '{key}' as written (raw_simple) is interpolated again through its result, unless that result is
// an int / float / bool / None value; such items report IE_RECURSE (W.recurse) and the caller
// walks them. Status and entry flags of a final result -> does recursive_interpolate re-enter it?
__device__ __forceinline__ bool recurses(uint8_t st, uint32_t flags) {
  const uint32_t k = flags & EF_KIND_MASK;
  return st == IE_OK_STR || (st == IE_OK_VALUE && (k == IE_KIND_STR || k == IE_KIND_LIST || k == IE_KIND_DICT));
}

// may the string (as written) be get_simple_insertkey-truthy (py:477-495)? Necessary conditions
// only: at least 3 bytes, and a '{' first or a '}' right after the first character (the depth must
// leave 0 at the second character). Any address space.
__device__ __forceinline__ bool maybe_simple(const uint8_t* s, uint32_t n) {
  if (n < 3) return false;
  const uint8_t c0 = s[0];
  if (c0 == '{') return true;
  const uint32_t l = c0 < 0x80u ? 1u : (c0 & 0xE0u) == 0xC0u ? 2u : (c0 & 0xF0u) == 0xE0u ? 3u : 4u;
  return l < n && s[l] == '}';
}

// The deferred tiles' bytes (see k_resolve): one workgroup per deferred tile at a time. Each
// lane rebuilds its string's pieces from the stored descriptor (template runs from the input in
// global memory, values from the table or the literal pool) and the tile's output goes through
// the LDS stage in windows of kRStageBytes (long pieces copied by a whole wave).
// One launch serves a whole call: the defer list holds the tiles of the batch B0 and, flagged
// kDeferSub, those of its deferred subset B1 (a two-pass views call: one emit after both passes).
constexpr uint32_t kDeferSub = 1u << 31;
__global__ __launch_bounds__(kRBlock) void k_emit_windows(Batch B0, Batch B1, Work W, DevTable T, uint8_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t s_win[kRStageBytes + 48];
  const uint32_t count = __hip_atomic_load(W.defer_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t tid = threadIdx.x;
  // views output: the bytes every tile claimed are the batch's total (k_resolve has finished)
  if (B0.out_len && blockIdx.x == 0 && tid == 0) {
    uint64_t t = 0;  // reserved ranges: the tiles' sums (the cursor counts the overflow region only)
    if (W.reserve16)
      for (uint32_t k = 0; k < 16; k++) t += W.shards[16u * k];
    *W.total = W.reserve16 ? t : *W.cursor;
  }
  // the call's telemetry straight into the host's pinned words (every resolve pass has finished)
  // (words 4-9: the five telemetry words and the windowed-tile count)
  if (W.stat_out && blockIdx.x == 0 && tid < 6) gst(W.stat_out + tid, tid < 5 ? W.stats[tid] : count);
  // the pool's demand: every resolve pass of the call has finished
  if (W.pool_out && blockIdx.x == 0 && tid == 0) {
    const uint64_t u = __hip_atomic_load(W.pool_used, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    gst(W.pool_out, (uint64_t)(((uint64_t)W.pool_seq << 40) | (u < (1ull << 40) ? u : (1ull << 40) - 1)));
  }
  // the next call's counters (the set this call did not use)
  if (W.zero_next && blockIdx.x == gridDim.x - 1)
    for (uint32_t k = tid; k < W.zero_words; k += kRBlock) gst(W.zero_next + k, 0u);
  // fewer deferred tiles than workgroups: each tile's windows are shared by `per` workgroups (a
  // tile of multi-KB outputs is hundreds of windows: one workgroup alone would take them in turn)
  const uint32_t per = count && count < gridDim.x ? gridDim.x / count : 1u;
  const uint32_t slot0 = per > 1u ? blockIdx.x / per : blockIdx.x, wk = per > 1u ? blockIdx.x % per : 0u;
  const uint32_t slot_step = per > 1u ? count : gridDim.x;  // (per > 1: one slot per workgroup)
  for (uint32_t slot = slot0; slot < count; slot += slot_step) {
    // the tile's record {tile | kDeferSub, -, base, total} and each lane's descriptor {.., local,
    // length}, as its k_resolve left them: a later pass of the same call may have rewritten the
    // batch's offsets / lengths / statuses of strings it deferred (its own results)
    const uint4 rec = gld4((const uint4*)(W.defer_tiles + 8ull * slot)), rec2 = gld4((const uint4*)(W.defer_tiles + 8ull * slot) + 1);
    const uint32_t tile = rec.x & ~kDeferSub;
    Batch B = (rec.x & kDeferSub) ? B1 : B0;  // (uniform)
    if (B.n_dev) {
      const uint64_t nd = gld(B.n_dev);
      B.n = nd < B.n ? nd : B.n;
    }
    const uint64_t first = (uint64_t)tile * kRBlock, i = first + tid;
    const uint64_t base = ((uint64_t)rec.w << 32) | rec.z;
    const uint64_t tile_total = ((uint64_t)rec2.y << 32) | rec2.x;
    const uint4* dd = W.defer_desc + ((uint64_t)slot * kRBlock + tid) * 4;
    Desc d;
    uint32_t olen = 0, n32 = 0;
    uint64_t local = 0;
    const uint8_t* s = B.bytes;
    if (i < B.n) {
      const uint4 a = gld4(dd), b = gld4(dd + 1), c = gld4(dd + 2), e = gld4(dd + 3);
      d.ntop = a.x, d.open[0] = a.y, d.open[1] = a.z, d.open[2] = a.w;
      d.close[0] = b.x, d.close[1] = b.y, d.close[2] = b.z, n32 = b.w;
      d.vk[0] = c.x, d.vk[1] = c.y, d.vk[2] = c.z;
      d.vs[0] = e.x, d.vs[1] = e.y, d.vs[2] = e.z;
      local = c.w;
      olen = e.w;
      s = B.bytes + gld(B.in_off + i);
    } else {
      d.ntop = 0;
#pragma unroll
      for (int q = 0; q < kMaxTop; q++) d.open[q] = d.close[q] = d.vk[q] = d.vs[q] = 0;
    }
    const bool mine = olen != 0;
    lds_u8* const win = (lds_u8*)s_win;
    for (uint64_t w0 = (uint64_t)wk * kRStageBytes; w0 < tile_total; w0 += (uint64_t)per * kRStageBytes) {
      const uint32_t wl = (uint32_t)min((uint64_t)kRStageBytes, tile_total - w0);
      const int64_t rel0 = (int64_t)local - (int64_t)w0;  // this lane's output, window-relative
      const bool on = mine && rel0 < (int64_t)wl && rel0 + (int64_t)olen > 0;
      const uint32_t ntop = mine ? d.ntop : 0u;
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j <= kMaxTop; j++) {
        const uint32_t t_lo = j == 0 ? 0u : d.close[j - 1] + 1;
        const uint32_t t_hi = (uint32_t)j < ntop ? d.open[j] : n32;
        const uint32_t tl = on && (uint32_t)j <= ntop ? t_hi - t_lo : 0u;
        window_piece<false>(win, rel0 + w, s + t_lo, tl, wl);
        w += tl;
        if (j == kMaxTop) break;
        const bool von = on && (uint32_t)j < ntop;
        const uint32_t kind = d.vk[j] >> 30, len = von ? d.vk[j] & kLenMask : 0u;
        const uint8_t* p = kind == kValEntry ? T.entries[von ? d.vs[j] : 0u].text
                           : kind == kValArena ? T.arena + d.vs[j]
                                               : W.pool + ((uint64_t)d.vs[j] << 4);
        window_piece<false>(win, rel0 + w, p, len, wl);
        w += len;
      }
      __syncthreads();
      stream_stage(out + base + w0, s_win, wl, tid);
      __syncthreads();
    }
  }
}

// FAILC: chain failures commit in the chain evaluator (else they take the exact evaluator). Both
// give the reference's results; the host picks per batch stream (ie_host.cpp, "fail commit").
// VIEWS: B.out_len set; each tile claims its output range with one atomic on W.cursor (no
// global order, no look-back) and writes each string's start and length.
// UNESC (with VIEWS): the unescape command's resolve, fused with its recursive_unescape: each
// staged string is unescaped in place in the LDS stage (after the classification; its chunks are
// classified again) and then resolved; strings that cannot be finished there (not staged, or
// needing the literal path) go to W.udefer_list for the deferred pass.
// SUB: a views deferred subset's instance, the only one with the grid-stride loop over tiles (in the
// others the loop's back edge made the compiler keep the prefetch and the entry-text registers in
// scratch: 53 spill stores and 80 reloads per tile in the views instance of scalar calls)
template <bool FAILC, bool MULTI, bool VIEWS, bool UNESC = false, bool LK = false, bool LEAN = false, bool SUB = false>
__global__ __launch_bounds__(kRBlock) __attribute__((amdgpu_waves_per_eu(
    LEAN && IE_LEAN5 ? IE_WAVES_PER_EU_LEAN : LK ? IE_WAVES_PER_EU_LK : IE_WAVES_PER_EU))) void k_resolve(Batch B0, Work W, DevTable T, uint8_t* out,
                                                    uint64_t cap) {
  constexpr bool L5 = LEAN && IE_LEAN5 != 0;
  // a deferred subset counts its strings on the device (the grid is sized for B0.n)
  Batch B = B0;
  if (B0.n_dev) {
    const uint64_t nd = gld(B0.n_dev);
    B.n = nd < B0.n ? nd : B0.n;
  }
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kRTileBytes + 48];
  __shared__ __attribute__((aligned(16))) uint8_t s_u[L5 ? kUnionLean : kUnionLds];
  __shared__ uint32_t s_olen[kRBlock];  // output length; the value id for IE_OK_VALUE strings
  __shared__ uint8_t s_st[kRBlock];
  __shared__ uint16_t s_pend[LEAN ? 1 : kRBlock];  // (no literal path in a LEAN pass)
  __shared__ uint16_t s_pil[LEAN && !L5 ? kLdsPilots : 1];  // a small table's pilots (LEAN)
// (measured slower, off: profiles/r06/lds_pilots/README.md)
#ifndef IE_LDS_PILOTS
#define IE_LDS_PILOTS 0
#endif
  const bool pil_lds = IE_LDS_PILOTS && LEAN && !L5 && T.nb <= kLdsPilots;
  __shared__ uint32_t s_misc[4];  // tile, pending count, defer slot
  __shared__ uint64_t s_red[kRBlock / 64 + 2];
  lds_u32* const s_cm = (lds_u32*)(lds_u8*)(s_u + (L5 ? kLCmOff : kCmOff));    // event masks of the staged chunks (+ pad)
  lds_u32* const s_odd = (lds_u32*)(lds_u8*)(s_u + (L5 ? kLOddOff : kOddOff));  // one bit per chunk: 0xE3 inside
  lds_u32* const s_esc = (lds_u32*)(lds_u8*)(s_u + (L5 ? kLEscOff : kEscOff));  // one bit per chunk: '\' inside
  lds_u32* const s_lit = (lds_u32*)(lds_u8*)s_u;              // literal-path results: pool offset >> 4

  const uint32_t tid0 = threadIdx.x;
  const uint32_t ntiles = (uint32_t)((B.n + kRBlock - 1) / kRBlock);
  // Views: tile = workgroup index (no tile waits on another). Packed output: the tile index is a
  // ticket taken when the workgroup starts, so every tile a look-back waits on has started (HIP
  // promises no dispatch order; one atomic per tile, on the packed path only)
  uint32_t tile = blockIdx.x;
  if (!VIEWS) {
    if (tid0 == 0) s_misc[0] = atomicAdd(W.tile_ticket, 1u);
    __syncthreads();
    tile = s_misc[0];
  }
  // a deferred subset (B0.n_dev: its string count is only known on the device) runs on a bounded
  // grid that strides over the tiles (a subset with nothing in it costs a few workgroups, not a
  // whole batch's: the SUB instances); every other launch has a workgroup per tile, one trip
  for (;;) {
  // (SUB: the lane index opaque per tile, so that nothing derived from it is kept in registers (or
  // scratch) across the loop's back edge; a no-op for the one-trip instances)
  uint32_t tid_l;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid_l) : "v"(tid0));
  const uint32_t tid = SUB ? tid_l : tid0, wave = tid >> 6, lane = tid & 63u;
  const TileGeo geo = load_geo(B, tile, tid);
  TilePrefetch<kStageV> pre;
  pre.nv = 0;
  if (tile < ntiles) pre.issue(B, geo, tid);
  // a small table's pilots, loaded with the tile's input (in flight together; stored to LDS with it)
  uint32_t pil0 = 0, pil1 = 0;
  if (pil_lds && tile < ntiles) {
    if (tid < T.nb) pil0 = gld(T.pilots + tid);
    if (tid + kRBlock < T.nb) pil1 = gld(T.pilots + tid + kRBlock);
  }
  if (tile < ntiles) {
  uint64_t t_start = 0;
  if (tid == 0) {
    if (W.stamps) t_start = __builtin_amdgcn_s_memrealtime();
    s_misc[1] = 0;
  }
  // diagnostic phase stamps (100 MHz s_memrealtime), one row of 16 words per tile
  uint64_t* const stamp_row = W.stamps ? W.stamps + (uint64_t)tile * 16 : nullptr;
#define IE_STAMP(k)                                                                  \
  do {                                                                               \
    if (stamp_row && tid == 0) stamp_row[k] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
  if (stamp_row && tid == 0) {
    stamp_row[0] = t_start;
    uint32_t hw = 0, xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    stamp_row[7] = ((uint64_t)xcc << 32) | hw;
  }
  const uint64_t first = (uint64_t)tile * kRBlock;
  const uint64_t last = min(first + (uint64_t)kRBlock, B.n);
  const uint64_t i = first + tid;
  const uint64_t lo = geo.lo, so = geo.so;
  uint64_t sn = geo.sn;
  const uint32_t shift = (uint32_t)((uintptr_t)(B.bytes + lo) & 15);
  // the stage holds the tile's first kStageChunks 16-byte chunks: strings that end inside it are
  // evaluated from LDS, the rest (a tile of long strings; a views input string placed apart from
  // its tile) from global memory
  const uint32_t nv = pre.nv;
  uint32_t p0 = shift + (uint32_t)(so - lo);
  const bool lane_staged = p0 + sn <= 16ull * nv;
  {
    pre.commit((uint4*)s_in, tid);
    if (pil_lds) {  // (uniform; their first reader is behind the classification's barriers)
      s_pil[tid] = (uint16_t)pil0;
      if (tid + kRBlock < kLdsPilots) s_pil[tid + kRBlock] = (uint16_t)pil1;
    }
    if (UNESC) {
      // the fused unescape command: per staged chunk, the bytes that are '\\' (bits 0-15) and the
      // braces (bits 16-31), from the prefetch registers, in the chunk-mask array (the
      // classification below overwrites it)
#pragma unroll
      for (int k = 0; k < kStageV; k++) {
        const uint32_t c = tid + (uint32_t)k * kRBlock;
        if (c < pre.nv) {
          const uint32_t w4[4] = {pre.v[k].x, pre.v[k].y, pre.v[k].z, pre.v[k].w};
          uint32_t bs = 0, br = 0;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint32_t x = w4[q], x7 = x & 0x7F7F7F7Fu;
            const uint32_t nb = ((x7 ^ 0x5C5C5C5Cu) + 0x7F7F7F7Fu) | x;
            const uint32_t no = ((x7 ^ 0x7B7B7B7Bu) + 0x7F7F7F7Fu) | x;
            const uint32_t nc = ((x7 ^ 0x7D7D7D7Du) + 0x7F7F7F7Fu) | x;
            bs |= nib(~nb) << (4 * q);
            br |= nib(~(no & nc)) << (4 * q);
          }
          s_cm[c] = bs | (br << 16);
        }
      }
      if (tid < 2) s_cm[pre.nv + tid] = 0;  // (the chunk after the last: no brace)
    }
    __syncthreads();
    if (UNESC) {
      // recursive_unescape (py:1436-1440, runtime.rs:1046: '\\{' -> '{', then '\\}' -> '}'; a
      // removed '\\' leaves a brace behind the byte before it, never a new pair, so one
      // left-to-right pass equals the two replaces; a '\\' that ends its string stays, the brace
      // after it being the next string's) on this lane's staged string, in place, before the
      // classification: only strings with a '\\' before a brace inside them have anything to do
      bool esc_in = false;
      if (lane_staged && sn > 1) {
        const uint32_t a = p0, z = p0 + (uint32_t)sn - 2u;  // candidate positions: not the last byte
        for (uint32_t c = a >> 4; c <= (z >> 4) && !esc_in; c++) {
          const uint32_t m = s_cm[c], mn = s_cm[c + 1];
          const uint32_t brn = (m >> 17) | ((mn >> 16) & 1u) << 15;  // brace at the next byte
          uint32_t d = m & 0xFFFFu & brn;
          if (c == (a >> 4)) d &= 0xFFFFu << (a & 15u);
          if (c == (z >> 4)) d &= 0xFFFFu >> (15u - (z & 15u));
          esc_in = d != 0u;
        }
      }
      uint32_t nsn = (uint32_t)sn;
      // the wave takes such strings one at a time, 64 bytes per step: a byte is kept unless it is
      // a '\\' before a brace; the kept bytes move down to their rank (in place: a step writes
      // only below its own block, which every lane has read)
      for (uint64_t todo = __ballot(esc_in); todo; todo &= todo - 1ull) {
        const uint32_t j = (uint32_t)__builtin_ctzll(todo);
        const uint32_t jp0 = (uint32_t)__shfl((int)p0, (int)j, 64), jsn = (uint32_t)__shfl((int)(uint32_t)sn, (int)j, 64);
        lds_u8* const b = (lds_u8*)s_in + jp0;
        uint32_t w = 0;
        for (uint32_t k0 = 0; k0 < jsn; k0 += 64) {
          const uint32_t k = k0 + lane;
          const uint8_t ch = k < jsn ? b[k] : (uint8_t)0;
          const uint8_t nx = k + 1u < jsn ? b[k + 1u] : (uint8_t)0;
          const bool keep = k < jsn && !(ch == '\\' && (nx == '{' || nx == '}'));
          const uint64_t km = __ballot(keep);
          if (keep) b[w + (uint32_t)__popcll(km & ((1ull << lane) - 1ull))] = ch;
          w += (uint32_t)__popcll(km);
        }
        if (lane == j) nsn = w;
      }
      sn = nsn;
      __syncthreads();  // every string's bytes are final: the classification sees the unescaped stage
    }
    for (uint32_t c0 = 0; c0 < nv; c0 += kRBlock) {  // uniform trip count: ballots below
      const uint32_t c = c0 + tid;
      bool odd = false, esc = false;
      if (c < nv) s_cm[c] = chunk_classify((const lds_u32*)(lds_u8*)s_in + 4 * c, odd, esc);
      const uint64_t ob = __ballot(odd), eb = __ballot(esc);
      if (lane == 0) {  // 64 consecutive chunks = two words of each bit array
        s_odd[(c0 + 64 * wave) >> 5] = (uint32_t)ob;
        s_odd[((c0 + 64 * wave) >> 5) + 1] = (uint32_t)(ob >> 32);
        s_esc[(c0 + 64 * wave) >> 5] = (uint32_t)eb;
        s_esc[((c0 + 64 * wave) >> 5) + 1] = (uint32_t)(eb >> 32);
      }
    }
    if (tid < 10) s_cm[nv + tid] = 0;  // the event windows read past the last chunk
  }
  __syncthreads();
  IE_STAMP(1);

  // ---- 2. evaluate ----
  Desc d;
  d.ntop = 0;
#pragma unroll
  for (int q = 0; q < kMaxTop; q++) d.open[q] = d.close[q] = d.vk[q] = d.vs[q] = 0;
  const uint8_t* s = nullptr;
  bool pend = false, chain_fail = false;
  // this string's table in the set (MULTI: a table-id batch; else every key lives in table 0)
  const uint32_t tid_s = (MULTI && i < B.n) ? gld(B.table_id + i) : 0u;
  {
    uint8_t st = IE_OK_STR;
    uint32_t olen = 0, vid = IE_VID_NONE, vflags = 0;
    bool active = false;
    if (i < B.n) {
      s = lane_staged ? s_in + p0 : B.bytes + so;
      // the unescape command (W.recurse): an item that may be a whole-string '{key}' as written
      // goes to the literal path, which decides IE_RECURSE with the whole wave (rare: a '{' first,
      // or a '}' right after the first character)
      active = sn < 0xFFFF0000ull && !(W.recurse && maybe_simple(s, (uint32_t)sn)) && (!UNESC || lane_staged);
      if (!active) st = kStatusPending;
    }
    uint8_t r = IE_OK_STR;
    bool slow = active;
    if (W.debug_noeval & 1u) {  // diagnostic: copy verbatim (the pipeline floor)
      olen = (uint32_t)sn;
      slow = false;
    } else if (W.fast_mode) {
      // chains: parse per string, resolve per chain job (tile-wide), gather per string. The job
      // arrays live in the union (results and string starts in the exact evaluator's key area,
      // records in the chunk masks once every string has read its event windows).
      uint32_t crec[kMaxTop], cdep[kMaxTop], nch = 0;
      Ev Om, Cm;
      uint32_t maxd;
      bool whole1;
      const bool pok = parse_chains((const lds_u8*)s_in, p0, (uint32_t)sn, s_cm, s_odd, s_esc, active && lane_staged,
                                    crec, cdep, nch, Om, Cm, maxd, whole1);
      if (!L5 && __any(maxd > 2u)) {  // middle levels are found from these masks in their round
        lds_u64* const ev = (lds_u64*)(lds_u8*)(s_u + kKbufLds) + tid;
        ev[0] = Om.lo, ev[kRBlock] = Om.hi, ev[2 * kRBlock] = Cm.lo, ev[3 * kRBlock] = Cm.hi;
      }
      uint64_t njobs64;
      // (its barrier: every wave has read the chunk masks the job records overwrite; the records'
      // barrier below comes before s_red is written again)
      const uint32_t jb = (uint32_t)block_scan<IE_FEWER_BARRIERS == 0>(pok ? nch : 0u, s_red, &njobs64);
      const uint32_t njobs = (uint32_t)njobs64;
      IE_STAMP(8);
      const ChainJobs J =
          L5 ? ChainJobs{(lds_u32*)(lds_u8*)(s_u + kLCrecOff), (lds_u16*)(lds_u8*)(s_u + kLMetaOff),
                         (lds_u32*)(lds_u8*)(s_u + kLCrecOff),  // (a job's result over its record)
                         (lds_u32*)(lds_u8*)(s_u + kLResSOff), (lds_u16*)(lds_u8*)(s_u + kLP0Off),
                         (lds_u32*)(lds_u8*)s_olen, nullptr, s_cm, s_odd, s_esc, nullptr}
             : ChainJobs{(lds_u32*)(lds_u8*)(s_u + kCmOff), (lds_u16*)(lds_u8*)(s_u + 8 * kJobCap),
                         (lds_u32*)(lds_u8*)s_u, (lds_u32*)(lds_u8*)(s_u + 4 * kJobCap),
                         (lds_u16*)(lds_u8*)(s_u + 10 * kJobCap), (lds_u32*)(lds_u8*)s_olen,
                         (lds_u64*)(lds_u8*)(s_u + kKbufLds), nullptr, nullptr, nullptr,
                         pil_lds ? (const lds_u16*)s_pil : nullptr};
      if (pok) {
#pragma unroll
        for (int c = 0; c < kMaxTop; c++) {
          if ((uint32_t)c < nch) {
            J.crec[jb + c] = crec[c];
            J.meta[jb + c] = (uint16_t)(tid | (cdep[c] << 12) | (whole1 ? 0x8000u : 0u));
          }
        }
      }
      J.p0[tid] = (uint16_t)p0;
      J.tbl[tid] = tid_s;
      __syncthreads();
      IE_STAMP(9);
      for (uint32_t j0 = 0; j0 < njobs; j0 += kJobsPerLaneOf<LK, L5> * kRBlock) resolve_jobs<FAILC, LK, L5>(T, (const lds_u8*)s_in, J, j0, njobs, chain_fail, j0 == 0 ? stamp_row : nullptr);
      IE_STAMP(10);
      __syncthreads();
      IE_STAMP(11);
      // (the fail-commit LEAN instances read the records back from LDS: they spilled otherwise, 20-24 B
      // per lane, config 4 1.420 -> 1.378 ms; the others keep them in registers, 1 % faster)
      const bool fast = pok && combine_chains<!L5 && LEAN && FAILC>(J, jb, nch, crec, (uint32_t)sn, d, olen, r, vid, vflags);
      __syncthreads();  // the job arrays are free (the exact evaluator's scratch)
      IE_STAMP(12);
      slow = active && !fast;
    }
    const uint64_t fail_m = __ballot(chain_fail);
    if (fail_m && lane == 0) atomicAdd(W.stats + 4, (uint32_t)__popcll(fail_m));  // misses: rare
    // a views batch with heavy strings (W.defer_slow, chosen per batch by the host): the strings the
    // chain jobs could not finish go to a second pass, in tiles of their own, instead of holding up
    // this tile (and its 255 other strings) in the exact evaluator or the literal path
    // LEAN (a views first pass, launch_resolve_deferring): this instance has no exact evaluator and
    // no literal path at all, so its registers and schedule are the chain evaluator's alone (config 3
    // 0.840 -> 0.804 ms, profiles/r05/ab/); every string they would take is deferred
    const bool dslow = VIEWS && !UNESC && (LEAN || W.defer_slow != 0u);
    if (dslow) {
      const uint64_t dm = __ballot(slow);
      if (dm && lane == 0) atomicAdd(W.stats + 3, (uint32_t)__popcll(dm));
      if (slow) r = kStatusDeferred;
      slow = false;
    }
    // the rest: the exact evaluator (scratch: the lane's own chain-evaluator columns)
    const uint64_t slow_m = LEAN ? 0ull : __ballot(slow);
    if (!LEAN && slow_m) {
      if (lane == 0 && W.fast_mode) atomicAdd(W.stats + 3, (uint32_t)__popcll(slow_m));  // rare
      lds_u8* const kb = (lds_u8*)(s_u + tid * kKeyCap);
      lds_u32* const stk = (lds_u32*)(lds_u8*)(s_u + kKbufLds) + tid;
      uint32_t o2 = 0;
      uint8_t r2 = kStatusPending;
#ifndef IE_EXP_NOEXACT
      // staged strings through a generic pointer into the stage, the rest in global memory
      r2 = eval_exact<false>(T, tid_s, Src<false>{s}, (uint32_t)sn, slow, kb, stk, d, o2, vid, vflags, W.err_keys != 0u);
#endif
      if (slow) r = r2, olen = o2;
    }
    if (active) st = r;
    if ((UNESC || dslow) && i < B.n && st == kStatusPending) {
      // the fused unescape command finishes in the stage only: the rest goes to the deferred pass
      // (so do the literal-path strings of a deferring views batch)
      st = kStatusDeferred;
    }
    if (UNESC || dslow) {
      const bool dfr = i < B.n && st == kStatusDeferred;
      const uint64_t m = __ballot(dfr);
      if (m) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(W.udefer_count, (uint32_t)__popcll(m));
        base = __shfl(base, 0, 64);
        const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (dfr) W.udefer_list[pos] = (uint32_t)i;
        if (LEAN && dfr) {  // (the second pass's view of the string: no gather kernel)
          // (the string's offset read again here, not held in registers across the chain jobs: the
          // fail-commit LEAN instance spilled it)
          W.sub_off[pos] = gld(B.in_off + i);
          W.sub_len[pos] = (uint32_t)min(sn, (uint64_t)0xFFFFFFFFu);
          if (MULTI) W.sub_tid[pos] = tid_s;
        }
      }
    }
    pend = !LEAN && i < B.n && st == kStatusPending;
    if (pend) s_pend[atomicAdd(&s_misc[1], 1u)] = (uint16_t)tid;
    s_st[tid] = st;
    s_olen[tid] = st == IE_OK_STR ? olen : (st == IE_OK_VALUE || st == IE_RECURSE ? vid : 0u);
  }
  __syncthreads();
  IE_STAMP(2);

  // ---- 3. literal path for the pending strings, one wave each; results in the union ----
  const uint32_t npend = LEAN ? 0u : s_misc[1];
  if (!LEAN && npend) {  // uniform
  if (tid == 0) atomicAdd(W.stats, npend);
  // the descriptors wait in the free part of the union while the waves run the literal path (its
  // registers are what the wave then needs; s_lit uses the union's first 4 * kRBlock bytes)
  lds_u32* const park = (lds_u32*)(lds_u8*)(s_u + 4 * kRBlock) + tid;
  park[0] = d.ntop;
#pragma unroll
  for (int q = 0; q < kMaxTop; q++) {
    park[(1 + q) * kRBlock] = d.open[q];
    park[(4 + q) * kRBlock] = d.close[q];
    park[(7 + q) * kRBlock] = d.vk[q];
    park[(10 + q) * kRBlock] = d.vs[q];
  }
  for (uint32_t k = wave; k < npend; k += kRBlock / 64) {
    const uint32_t j = s_pend[k];
    const uint64_t gi = first + j;
    const uint64_t po = gld(B.in_off + gi), pn = in_length(B, gi);
    uint64_t rcap = W.lit_cap_max ? IE_SIZE_CAP(pn, T.maxtext) + 4 * T.maxtext + 64
                                  : 4 * pn + 4 * T.maxtext + 256;
    rcap = pn >= 0xFFFF0000ull ? 0ull : (rcap + 15) & ~15ull;  // (a string the pool never took: overflow)
    uint64_t pbase = 0;
    if (lane == 0) pbase = atomicAdd((unsigned long long*)W.pool_used, (unsigned long long)(4 * rcap));
    pbase = __shfl(pbase, 0, 64);
    LitOut r{IE_E_OVERFLOW, 0, 0, IE_VID_NONE, 0, nullptr, 0};
#ifndef IE_EXP_NOLIT
    if (rcap && pbase + 4 * rcap <= W.pool_bytes)
#else
    if (false)
#endif
      r = w_literal(T, MULTI ? gld(B.table_id + gi) : 0u, B.bytes + po, pn, W.pool + pbase, rcap, pbase,
                    W.lit_cap_max != 0);
    if (r.status == IE_OK_STR && (r.res_len > kLenMask || (r.res_off >> 4) > 0xFFFFFFFFull))
      r.status = IE_E_OVERFLOW;
    if ((r.status == IE_NEEDS_HOST || (W.err_keys && r.status == IE_E_INTERP)) && W.host_keys && r.key) {
      // the key the host must look up (get_interpdata's file fallback, py:452-461), or the missing
      // key an IE_E_INTERP message names (py:467): a record {string index, key length, key bytes}
      // in the exec's host-key list
      const uint64_t need = 8 + ((r.key_len + 3ull) & ~3ull);
      uint64_t at = 0;
      if (lane == 0) at = atomicAdd((unsigned long long*)W.host_keys_used, (unsigned long long)need);
      at = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(at >> 32), 0, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)at, 0, 64);
      if (at + need <= W.host_keys_cap) {
        if (lane == 0) {
          uint32_t* hdr = (uint32_t*)(W.host_keys + at);
          hdr[0] = B.out_index ? gld(B.out_index + gi) : (uint32_t)gi;
          hdr[1] = r.key_len;
        }
        for (uint32_t k = lane; k < r.key_len; k += 64) W.host_keys[at + 8 + k] = r.key[k];
      }
    }

    if (lane == 0) {
      uint64_t ko, kl;  // W.recurse: get_simple_insertkey on the item as written (py:1463)
      const uint8_t* const item = B.bytes + po;
      if (W.recurse && recurses(r.status, r.flags) &&
          simple_insertkey([item](uint64_t k) { return item[k]; }, pn, 0u, ko, kl)) {
        if (r.status == IE_OK_STR) r.vid = IE_VID_NONE;
        r.status = IE_RECURSE;
      }
      s_st[j] = r.status;
      s_olen[j] = r.status == IE_OK_STR ? (uint32_t)r.res_len : (r.status == IE_OK_VALUE || r.status == IE_RECURSE ? r.vid : 0u);
      s_lit[j] = (uint32_t)(r.res_off >> 4);
    }
  }
  d.ntop = park[0];
#pragma unroll
  for (int q = 0; q < kMaxTop; q++) {
    d.open[q] = park[(1 + q) * kRBlock];
    d.close[q] = park[(4 + q) * kRBlock];
    d.vk[q] = park[(7 + q) * kRBlock];
    d.vs[q] = park[(10 + q) * kRBlock];
  }
  }
  if (!IE_FEWER_BARRIERS || npend) __syncthreads();  // (nothing was written since the last barrier otherwise)
  IE_STAMP(3);

  // ---- 4. offsets: workgroup scan; the aggregate goes out at once ----
  const uint8_t st = s_st[tid];
  const uint32_t olen = st == IE_OK_STR ? s_olen[tid] : 0u;
  const uint32_t n32 = (uint32_t)sn;
  if (pend) {  // a literal-path result: the whole output is one pool value
    d.ntop = 1;
    d.open[0] = 0;
    d.close[0] = n32 - 1u;
    d.vk[0] = (kValPool << 30) | olen;
    d.vs[0] = s_lit[tid];
  }
#if IE_EARLY_TEXT
  // value 0's entry text in flight across the scan's barriers (its latency no longer opens the build)
  const bool mine = i < B.n && st == IE_OK_STR && olen;
  uint32_t tt[2][8];
  auto load_text = [&](int j, uint32_t (&t)[8]) {
    const bool need = mine && (uint32_t)j < d.ntop && (d.vk[j] >> 30) == kValEntry;
    if (__any(need)) {
      const uint4* tp = (const uint4*)(T.entries + (need ? d.vs[j] : 0u)) + 2;
      const uint4 t2 = gld4(tp), t3 = gld4(tp + 1);
      t[0] = t2.x, t[1] = t2.y, t[2] = t2.z, t[3] = t2.w;
      t[4] = t3.x, t[5] = t3.y, t[6] = t3.z, t[7] = 0;
    }
  };
  load_text(0, tt[0]);
#endif
  uint64_t tile_total;
  // (its barrier also retires s_lit; s_red[kRBlock / 64] below is another word than the scan's)
  const uint64_t local = block_scan<IE_FEWER_BARRIERS == 0>(olen, s_red, &tile_total);
  uint64_t lb_early = 0;
  if (VIEWS) {
    // the tile's output range: one atomic, its answer consumed after the build; or (reserved
    // ranges) the tile's own part of the output, no atomic unless it overflows its reservation
    if (tid == 0) {
      if (W.debug_noeval & 2u) {
        lb_early = 2 * lo;  // diagnostic: no claim (a range from the input's)
      } else if (W.reserve16) {
        // the reserved pass (packed input) computes the overflow region's start itself (two words
        // every tile reads: L2-resident) and tile 0 leaves it for later subset passes
        uint64_t rb = 0, ovf;
        bool own = false;
        if (!B.in_len && !B.out_index) {
          const uint64_t res_base = gld(B.in_off);
          ovf = ((((gld(B.in_off + B.n) - res_base) * W.reserve16) >> 4) + 15) & ~15ull;
          // (16-aligned: the stream-out then moves the stage's blocks as they are)
          rb = ((((lo - res_base) * W.reserve16) >> 4) + 15) & ~15ull;
          const uint64_t re = ((geo.hi - res_base) * W.reserve16) >> 4;
          own = rb <= re && tile_total <= re - rb;
          if (tile == 0) __hip_atomic_store(W.res_ovf, ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          ovf = __hip_atomic_load(W.res_ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        lb_early = own ? rb : ovf + atomicAdd((unsigned long long*)W.cursor, (unsigned long long)((tile_total + 15) & ~15ull));
        __hip_atomic_fetch_add(W.shards + 16u * (tile & 15u), tile_total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        lb_early = atomicAdd((unsigned long long*)W.cursor, (unsigned long long)tile_total);
      }
    }
  } else if (wave == 0) {
    publish_aggregate(W.tile_state, tile, tile_total);
    if (tile != 0) lb_early = lb_poll(W.tile_state, (int64_t)tile - 1);  // consumed after the build
  }

  // ---- 5. the tile's output bytes into the LDS stage (tile-relative offsets) while the
  //      look-back is pending; tiles whose output does not fit store straight to HBM later ----
  // (a fail-commit LEAN pass: the string's pointer made again here, not held in registers across
  // the chain jobs; a string past the stage reads its offset again)
  const uint8_t* const sx = !(LEAN && FAILC) ? s : i < B.n ? (lane_staged ? s_in + p0 : B.bytes + gld(B.in_off + i)) : nullptr;
  // (LEAN5: the output's first kLWin bytes go to the window stage (the union), the rest straight to
  // HBM; a tile of more than kLDirectMax bytes is deferred)
  const bool in_stage = L5 ? tile_total <= (uint64_t)kLDirectMax : tile_total <= (uint64_t)kOutStage;
#if !IE_EARLY_TEXT
  const bool mine = i < B.n && st == IE_OK_STR && olen;
#endif
  // LEAN5: the tile's place first (its bytes past the window are stored during the build)
  if (L5) {
    if (tid == 0) s_red[kRBlock / 64] = lb_early;
    __syncthreads();
  }
  const uint64_t base5 = L5 ? s_red[kRBlock / 64] : 0ull;
  // LEAN5: this lane's output in one pass over its pieces: the bytes in the window [0, kLWin) of
  // the tile's output to the window stage (template runs from the input stage, entry texts from
  // registers, arena texts by lane or by wave), the bytes past it stored straight to their place in
  // HBM by the lane (a piece across the edge: in part each way), so that no second build follows
  // the window's stream-out
  const uint32_t local_w = (uint32_t)local;
  uint8_t* const gout = out + base5;
  auto build_direct = [&]() {
    const lds_u8* const ls = (const lds_u8*)sx;
    const uint32_t ntop = mine ? d.ntop : 0u;
    const bool in_win = mine && local_w < kLWin;              // (bytes in the window)
    const bool past = mine && local_w + olen > kLWin;         // (bytes past it)
    uint32_t w = local_w;  // the next piece's place in the tile's output
    // 1. the window's bytes, and the entry texts wholly past it (from the registers)
#pragma unroll
    for (int j = 0; j <= kMaxTop; j++) {
      // template run j
      const uint32_t t_lo = j == 0 ? 0u : d.close[j - 1] + 1;
      const uint32_t t_hi = (uint32_t)j < ntop ? d.open[j] : n32;
      const uint32_t tl = mine && (uint32_t)j <= ntop ? t_hi - t_lo : 0u;
      const uint32_t tb = w + tl < kLWin ? w + tl : kLWin;
      const uint32_t tn = in_win && w < tb ? tb - w : 0u;
      if (__any(tn != 0)) {
        lds_u8* const dst = (lds_u8*)s_u + (tn ? w : 0u);
        if (lane_staged) lds_copy(dst, tn ? ls + t_lo : (const lds_u8*)s_in, tn);
        else if (tn) copy_bytes<true, false>((uint8_t*)dst, sx + t_lo, tn);  // a string past the stage
      }
      w += tl;
      if (j == kMaxTop) break;
      // value j
      if (j + 1 < kMaxTop) load_text(j + 1, tt[(j + 1) & 1]);
      const bool von = mine && (uint32_t)j < ntop;
      const uint32_t kind = d.vk[j] >> 30, len = von ? d.vk[j] & kLenMask : 0u;
      const bool ent = von && kind == kValEntry;
      const uint32_t vb = w + len < kLWin ? w + len : kLWin;
      const bool vin = von && w < vb;
      const bool ewhole = ent && vin && vb == w + len;
      if (__any(ewhole) && ewhole) put_words((lds_u8*)s_u + w, tt[j & 1], len);
      if (ent && vin && !ewhole) {  // (an entry text across the edge: its window part, byte by byte)
        const uint8_t* tx = T.entries[d.vs[j]].text;
        for (uint32_t k = w; k < vb; k++) ((lds_u8*)s_u)[k] = gld(tx + (k - w));
      }
      const bool far = vin && kind != kValEntry;  // an arena text
      if (__any(far))
        stage_piece((lds_u8*)s_u, far, far ? w : 0u, kind == kValArena ? T.arena + d.vs[j] : W.pool + ((uint64_t)d.vs[j] << 4),
                    far ? vb - w : 0u);
      const bool eg = ent && w >= kLWin;
      if (__any(eg) && eg) put_words_g(gout + w, tt[j & 1], len);
      w += len;
    }
    // 2. the rest past the window, by the lane (not unrolled: one copy loop of each kind): template
    //    runs from the input stage, arena texts and entry texts across the edge from the table
    if (__any(past)) {
      uint32_t pw = local_w;
#pragma unroll 1
      for (uint32_t j = 0; past && j <= ntop; j++) {
        const uint32_t t_lo = j == 0 ? 0u : d.close[j - 1] + 1;
        const uint32_t t_hi = j < ntop ? d.open[j] : n32;
        const uint32_t tl = t_hi - t_lo, ga = pw > kLWin ? pw : kLWin;
        if (ga < pw + tl) {
          if (lane_staged) copy_bytes<false, true>(gout + ga, (const uint8_t*)(ls + t_lo + (ga - pw)), pw + tl - ga);
          else copy_bytes<false, false>(gout + ga, sx + t_lo + (ga - pw), pw + tl - ga);
        }
        pw += tl;
        if (j == ntop) break;
        const uint32_t vk = j == 0 ? d.vk[0] : j == 1 ? d.vk[1] : d.vk[2];
        const uint32_t vs = j == 0 ? d.vs[0] : j == 1 ? d.vs[1] : d.vs[2];
        const uint32_t kind = vk >> 30, len = vk & kLenMask, va = pw > kLWin ? pw : kLWin;
        if (va < pw + len && !(kind == kValEntry && pw >= kLWin))  // (not an entry text wholly past: step 1's)
          copy_bytes<false, false>(gout + va,
                                   (kind == kValEntry ? (const uint8_t*)T.entries[vs].text
                                    : kind == kValArena ? T.arena + vs : W.pool + ((uint64_t)vs << 4)) + (va - pw),
                                   pw + len - va);
        pw += len;
      }
    }
  };
  if (L5) {
    if (in_stage && base5 + tile_total <= cap) build_direct();
  } else if (in_stage) {
    // entry texts of the values (inline, <= kInlineText bytes): into registers, value j's loads
    // issued one value ahead of its use
#if !IE_EARLY_TEXT
    uint32_t tt[2][8];
    auto load_text = [&](int j, uint32_t (&t)[8]) {
      const bool need = mine && (uint32_t)j < d.ntop && (d.vk[j] >> 30) == kValEntry;
      if (__any(need)) {
        const uint4* tp = (const uint4*)(T.entries + (need ? d.vs[j] : 0u)) + 2;
        const uint4 t2 = gld4(tp), t3 = gld4(tp + 1);
        t[0] = t2.x, t[1] = t2.y, t[2] = t2.z, t[3] = t2.w;
        t[4] = t3.x, t[5] = t3.y, t[6] = t3.z, t[7] = 0;
      }
    };
    load_text(0, tt[0]);
#endif
    lds_u8* const dd = (lds_u8*)(s_u + (mine ? local : 0));
    const lds_u8* const ls = (const lds_u8*)sx;
    const uint32_t ntop = mine ? d.ntop : 0u;
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j <= kMaxTop; j++) {
      // template run j
      const bool ton = mine && (uint32_t)j <= ntop;
      const uint32_t t_lo = j == 0 ? 0u : d.close[j - 1] + 1;
      const uint32_t t_hi = (uint32_t)j < ntop ? d.open[j] : n32;
      const uint32_t tl = ton ? t_hi - t_lo : 0u;
      if (__any(tl != 0)) {
        if (lane_staged) lds_copy(dd + w, tl ? ls + t_lo : (const lds_u8*)s_in, tl);
        else if (tl) copy_bytes<true, false>((uint8_t*)(dd + w), sx + t_lo, tl);  // a string past the stage
      }
      w += tl;
      if (j == kMaxTop) break;
      // value j
      if (j + 1 < kMaxTop) load_text(j + 1, tt[(j + 1) & 1]);
      const bool von = mine && (uint32_t)j < ntop;
      const uint32_t kind = d.vk[j] >> 30, len = von ? d.vk[j] & kLenMask : 0u;
      const bool ent = von && kind == kValEntry;
      if (__any(ent) && ent) put_words(dd + w, tt[j & 1], len);
      const bool far = von && kind != kValEntry;  // an arena or literal-pool text
      if (__any(far))
        stage_piece((lds_u8*)s_u, far, (uint32_t)(mine ? local : 0) + w,
                    kind == kValArena ? T.arena + d.vs[j] : W.pool + ((uint64_t)d.vs[j] << 4), len);
      w += len;
    }
  }
  IE_STAMP(4);
  if (VIEWS) {
    if (!L5 && tid == 0) s_red[kRBlock / 64] = lb_early;
  } else if (wave == 0) {
    const uint64_t b = look_back(W.tile_state, tile, tile_total, W.err, W.stamps ? W.stats + 2 : nullptr, lb_early);
    if (tid == 0) s_red[kRBlock / 64] = b;
  }
  __syncthreads();
  const uint64_t base = s_red[kRBlock / 64];
  // the lane index, opaque to the compiler from here on: the tail recomputes its indices instead
  // of keeping (and spilling) the staging loop's, which are equal expressions of threadIdx.x
  uint32_t tid_t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid_t) : "v"(tid));
  const uint64_t i_t = first + tid_t;
  if (i_t < B.n && !(W.debug_noeval & 8u)) {  // (diagnostic bit 3: no per-string stores, a traffic split)
    // (a deferred subset writes at its strings' places in the batch; a string the fused unescape
    // command deferred is written again by the deferred pass)
    const uint64_t o_i = B.out_index ? (uint64_t)gld(B.out_index + i_t) : i_t;
    gsts(B.out_off + o_i, base + local);
    if (VIEWS) gsts(B.out_len + o_i, s_st[tid_t] == IE_OK_STR ? s_olen[tid_t] : 0u);
    gsts(B.status + o_i, st);
    if (st == IE_OK_VALUE || st == IE_RECURSE) gst(B.value_id + o_i, s_olen[tid_t]);
  }
  if (!VIEWS && last == B.n && tid == 0) {
    B.out_off[B.n] = base + tile_total;
    *W.total = base + tile_total;
  }
  // views, one tile: the only claim on the cursor is this tile's, so the batch's total is its end
  // (k_emit_windows writes the same; a one-tile scalar call may skip that kernel)
  // (not in the LEAN first pass: its emit kernel always runs, and its code stays as it was)
  if (VIEWS && !LEAN && gridDim.x == 1u && !W.reserve16 && !(W.debug_noeval & 2u) && tid == 0) *W.total = base + tile_total;
  const bool write_bytes = base + tile_total <= cap;  // caller's buffer too small: offsets only
  // (reserved ranges: *total is the sum of lengths, not the extent, so the flag tells the caller)
  if (VIEWS && W.reserve16 && !write_bytes && tid == 0) atomicOr(W.err, 2u);

  // ---- 6. stream out: 16-byte stores at 16-byte aligned addresses, each assembled from the
  //      two stage blocks it straddles (the shift is uniform over the tile) ----
  uint8_t* const g = out + base;
  if (L5 && write_bytes && in_stage) {
    // the window (the bytes past it are out already)
    uint32_t tid_w;  // (opaque: the stream-out's per-block addresses computed here, not kept from before)
    asm volatile("v_mov_b32 %0, %1" : "=v"(tid_w) : "v"(tid_t));
    if (!(W.debug_noeval & 4u))  // (diagnostic bit 2: no bytes)
      stream_stage<kLWin>(g, s_u, (uint32_t)min((uint64_t)kLWin, tile_total), tid_w);
  } else if (!L5 && write_bytes && in_stage) {
    if (!(W.debug_noeval & 4u)) stream_stage(g, s_u, (uint32_t)tile_total, tid_t);  // (diagnostic bit 2: no bytes)
  } else if (write_bytes) {
    // a tile whose output exceeds the stage (long strings, large expansions) or whose input was
    // not staged: its descriptors go to the defer list and k_emit_windows writes its bytes
    // (offsets and statuses are final already); the windowed copy is kept out of this kernel so
    // that its registers do not weigh on the common path
    if (tid == 0) s_misc[2] = atomicAdd(W.defer_count, 1u);
    __syncthreads();
    const uint32_t slot = s_misc[2];
    uint4* dd = W.defer_desc + ((uint64_t)slot * kRBlock + tid_t) * 4;
    const uint32_t nt = mine ? d.ntop : 0u;
    gst4(dd, make_uint4(nt, d.open[0], d.open[1], d.open[2]));
    gst4(dd + 1, make_uint4(d.close[0], d.close[1], d.close[2], n32));
    gst4(dd + 2, make_uint4(d.vk[0], d.vk[1], d.vk[2], mine ? (uint32_t)local : 0u));
    gst4(dd + 3, make_uint4(d.vs[0], d.vs[1], d.vs[2], mine ? olen : 0u));
    if (tid == 0) {  // the tile's record (a subset's tile: flagged)
      uint4* r = (uint4*)(W.defer_tiles + 8ull * slot);
      gst4(r, make_uint4(tile | (B.out_index ? kDeferSub : 0u), 0u, (uint32_t)base, (uint32_t)(base >> 32)));
      gst4(r + 1, make_uint4((uint32_t)tile_total, (uint32_t)(tile_total >> 32), 0u, 0u));
    }
  }
  IE_STAMP(5);
#undef IE_STAMP
  }
  if (!SUB || !B0.n_dev) break;  // (uniform)
  tile += gridDim.x;
  if (tile >= ntiles) break;
  __syncthreads();  // the next tile's stage and union: every wave is done with this one's
  }
  // a one-tile host call without copies (W.ctr_host, ie_host.cpp run_host_small_zc; the launch is
  // this workgroup alone): the call's counter words to the host, then zeroed for its next call
  if (VIEWS && !LEAN && !SUB && !UNESC && W.ctr_host) {
    __threadfence();
    __syncthreads();  // (every access of this call to the counters is done)
    if (tid0 < 16u) {
      const uint32_t v = __hip_atomic_load(W.tile_ticket + tid0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      gst(W.ctr_host + tid0, v);
      __hip_atomic_store(W.tile_ticket + tid0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// diagnostic: one key through the device lookups. out[0..1] hash, out[2] slot, out[3] find_bytes,
// out[4] find_small (klen <= kInlineKey), out[5] entries, out[12] find_bytes by all 64 lanes,
// out[13] lane agreement ballot
__global__ void k_debug_probe(DevTable T, const uint8_t* key, uint32_t klen, uint64_t* out) {
  __shared__ uint32_t kb[16];
  const uint32_t lane = threadIdx.x;
  if (lane < 16) kb[lane] = 0;
  __syncthreads();
  if (lane == 0)
    for (uint32_t j = 0; j < klen && j < 64; j++) ((uint8_t*)kb)[j] = key[j];
  __syncthreads();
  Hit hw{0, 0, 0, 0};
  const int32_t fw = find_bytes(T, 0, key, klen, hw);
  const uint64_t agree = __ballot(fw == __shfl(fw, 0, 64) && hw.text_off == __shfl(hw.text_off, 0, 64));
  if (lane != 0) return;
  const uint64_t hash = hash_key(klen, [&](uint32_t j) { return key[j]; }, T.seed, 0u);
  Hit h;
  const int32_t fb = find_bytes(T, 0, key, klen, h);
  const int32_t fs = klen <= kInlineKey ? find_small(T, 0, (const uint32_t*)kb, klen, h) : -2;
  out[0] = hash & 0xFFFFFFFFull;
  out[1] = hash >> 32;
  out[2] = ph_lookup_slot(T, hash);
  out[3] = (uint64_t)(int64_t)fb;
  out[4] = (uint64_t)(int64_t)fs;
  out[5] = T.m;
  out[12] = (uint64_t)(int64_t)fw;
  out[13] = agree;
}

hipError_t launch_debug_probe_impl(const DevTable& T, const uint8_t* key, uint32_t klen, uint64_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_debug_probe, dim3(1), dim3(64), 0, st, T, key, klen, out);
  return hipGetLastError();
}

// the unescape command's deferred strings (see k_resolve<.., UNESC>): each block takes 256 entries
// of the deferred list, unescapes them (recursive_unescape, py:1665) into the literal pool with one
// claim per block (so the strings of a block lie together, in list order) and writes the views the
// deferred resolve reads; a string the pool cannot take gets the length that resolves to
// IE_E_OVERFLOW
__global__ __launch_bounds__(kRBlock) void k_unesc_deferred(Batch B, Work W, uint64_t* sub_off, uint32_t* sub_len,
                                                           uint32_t* sub_tid) {
  __shared__ uint64_t s_red[kRBlock / 64 + 2];
  const uint32_t count = __hip_atomic_load(W.udefer_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (uint64_t blk = blockIdx.x; blk * kRBlock < count; blk += gridDim.x) {
    const uint64_t j = blk * kRBlock + threadIdx.x;
    const bool on = j < count;
    uint32_t idx = 0;
    uint64_t so = 0, n = 0, un = 0;
    if (on) {
      idx = W.udefer_list[j];
      so = gld(B.in_off + idx);
      n = in_length(B, idx);
    }
    const uint8_t* const src = B.bytes + so;
    auto dropped = [&](uint64_t k) {  // '\\' before a brace of the same string
      return src[k] == '\\' && k + 1 < n && (src[k + 1] == '{' || src[k + 1] == '}');
    };
    for (uint64_t k = 0; k < n; k++) un += dropped(k) ? 0u : 1u;
    uint64_t tot;
    const uint64_t local = block_scan(un, s_red, &tot);
    if (threadIdx.x == 0)
      s_red[kRBlock / 64] = atomicAdd((unsigned long long*)W.pool_used, (unsigned long long)((tot + 15) & ~15ull));
    __syncthreads();
    const uint64_t base = s_red[kRBlock / 64];
    const bool fits = base + tot <= W.pool_bytes && un < 0xFFFF0000ull;
    if (on) {
      if (fits) {
        uint8_t* const dst = W.pool + base + local;
        uint64_t w = 0;
        for (uint64_t k = 0; k < n; k++)
          if (!dropped(k)) dst[w++] = src[k];
      }
      sub_off[j] = fits ? base + local : 0;
      sub_len[j] = fits ? (uint32_t)un : 0xFFFFFFFFu;
      if (sub_tid) sub_tid[j] = B.table_id ? gld(B.table_id + idx) : 0u;
    }
    __syncthreads();
  }
}

// the deferred subset's bounded grid (see k_resolve): 4 workgroups per CU
constexpr uint32_t kSubsetGrid = 1024;

// emit: launch k_emit_windows after the resolve (false: the caller launches one for the whole call,
// launch_emit)
hipError_t launch_resolve_impl(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                               hipStream_t st, bool unesc = false, bool lean = false, bool no_emit = false,
                               bool emit = true) {
  const uint64_t tiles = (B.n + kRBlock - 1) / kRBlock;
  if (!tiles) return hipSuccess;
  if (tiles > 0xFFFFFFFFull) return hipErrorInvalidValue;
  const uint32_t emax = W.emit_grid ? W.emit_grid : 512u, smax = W.sub_grid ? W.sub_grid : kSubsetGrid;
  const uint32_t egrid = (uint32_t)(tiles < emax ? tiles : emax);
  // (a subset views batch strides over its tiles: the SUB instances of k_resolve)
#if !defined(IE_RESOLVE_WIDE)
  const bool sub = B.n_dev && B.out_len && !unesc && !lean;
#else
  const bool sub = false;  // (the 512-string kernels never run a views subset: a whole grid if one did)
#endif
  const uint32_t grid = sub ? (uint32_t)(tiles < smax ? tiles : smax) : (uint32_t)tiles;
  const bool multi = B.table_id != nullptr;
#ifndef IE_EXP_ONLY_LEAN  // (experiments: -DIE_EXP_ONLY_LEAN compiles the LEAN instances alone, tools/resusage.sh)
  if (unesc) {  // the fused unescape command (views only)
    if (!B.out_len) return hipErrorInvalidValue;
    const int v = (W.fail_commit ? 2 : 0) | (multi ? 1 : 0);
    if (v == 0) hipLaunchKernelGGL((k_resolve<false, false, true, true>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap);
    if (v == 1) hipLaunchKernelGGL((k_resolve<false, true, true, true>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap);
    if (v == 2) hipLaunchKernelGGL((k_resolve<true, false, true, true>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap);
    if (v == 3) hipLaunchKernelGGL((k_resolve<true, true, true, true>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap);
    if (emit) hipLaunchKernelGGL(k_emit_windows, dim3(egrid), dim3(kRBlock), 0, st, B, B, W, T, out);
    return hipGetLastError();
  }
#endif
  // LK: a table with 17-32 byte keys gets the instances whose chain jobs take such keys (they cost
  // config 3 3 %: their registers; config 5 -32 %: its long keys leave the exact evaluator)
  const int variant = ((T.flags & TF_LONG_KEYS) ? 8 : 0) | (W.fail_commit ? 4 : 0) | (multi ? 2 : 0) | (B.out_len ? 1 : 0);
#if !defined(IE_RESOLVE_WIDE)
  if (lean && B.out_len) {  // the views first pass without the exact evaluator and literal path
    switch (variant >> 1) {
#define IE_LAUNCH_LEAN(V, F, M, L) \
  case V: hipLaunchKernelGGL((k_resolve<F, M, true, false, L, true>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap); break;
      IE_LAUNCH_LEAN(0, false, false, false)
      IE_LAUNCH_LEAN(1, false, true, false)
      IE_LAUNCH_LEAN(2, true, false, false)
      IE_LAUNCH_LEAN(3, true, true, false)
      IE_LAUNCH_LEAN(4, false, false, true)
      IE_LAUNCH_LEAN(5, false, true, true)
      IE_LAUNCH_LEAN(6, true, false, true)
      IE_LAUNCH_LEAN(7, true, true, true)
#undef IE_LAUNCH_LEAN
    }
    if (emit) hipLaunchKernelGGL(k_emit_windows, dim3(egrid), dim3(kRBlock), 0, st, B, B, W, T, out);
    return hipGetLastError();
  }
#endif
#if !defined(IE_EXP_ONLY_LEAN) && !defined(IE_RESOLVE_WIDE)
  if (sub) {
    switch (variant >> 1) {  // (views: bit 0 set)
#define IE_LAUNCH_SUB(V, F, M, L) \
  case V: hipLaunchKernelGGL((k_resolve<F, M, true, false, L, false, true>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap); break;
      IE_LAUNCH_SUB(0, false, false, false)
      IE_LAUNCH_SUB(1, false, true, false)
      IE_LAUNCH_SUB(2, true, false, false)
      IE_LAUNCH_SUB(3, true, true, false)
      IE_LAUNCH_SUB(4, false, false, true)
      IE_LAUNCH_SUB(5, false, true, true)
      IE_LAUNCH_SUB(6, true, false, true)
      IE_LAUNCH_SUB(7, true, true, true)
#undef IE_LAUNCH_SUB
    }
    if (emit && (out || B.out_len)) hipLaunchKernelGGL(k_emit_windows, dim3(egrid), dim3(kRBlock), 0, st, B, B, W, T, out);
    return hipGetLastError();
  }
#endif
#ifndef IE_EXP_ONLY_LEAN
  switch (variant) {
#define IE_LAUNCH(V, F, M, S, L) \
  case V: hipLaunchKernelGGL((k_resolve<F, M, S, false, L>), dim3(grid), dim3(kRBlock), 0, st, B, W, T, out, cap); break;
    IE_LAUNCH(0, false, false, false, false)
    IE_LAUNCH(1, false, false, true, false)
    IE_LAUNCH(2, false, true, false, false)
    IE_LAUNCH(3, false, true, true, false)
    IE_LAUNCH(4, true, false, false, false)
    IE_LAUNCH(5, true, false, true, false)
    IE_LAUNCH(6, true, true, false, false)
    IE_LAUNCH(7, true, true, true, false)
    IE_LAUNCH(8, false, false, false, true)
    IE_LAUNCH(9, false, false, true, true)
    IE_LAUNCH(10, false, true, false, true)
    IE_LAUNCH(11, false, true, true, true)
    IE_LAUNCH(12, true, false, false, true)
    IE_LAUNCH(13, true, false, true, true)
    IE_LAUNCH(14, true, true, false, true)
    IE_LAUNCH(15, true, true, true, true)
#undef IE_LAUNCH
  }
#endif
  // the deferred (oversized) tiles' bytes (exits at once when there are none); views: the total
  // (a one-tile views batch may go without it: no_emit, see launch_resolve)
  if (emit && (out || B.out_len) && !(no_emit && grid == 1u && B.out_len && !W.reserve16))
    hipLaunchKernelGGL(k_emit_windows, dim3(egrid), dim3(kRBlock), 0, st, B, B, W, T, out);
  return hipGetLastError();
}

// one k_emit_windows for a call of two passes: the batch B and its deferred subset D
hipError_t launch_emit(const Batch& B, const Batch& D, const Work& W, const DevTable& T, uint8_t* out,
                       hipStream_t st) {
  const uint64_t tiles = (B.n + kRBlock - 1) / kRBlock;
  if (!tiles) return hipSuccess;
  const uint32_t emax = W.emit_grid ? W.emit_grid : 512u;
  hipLaunchKernelGGL(k_emit_windows, dim3((uint32_t)(tiles < emax ? tiles : emax)), dim3(kRBlock), 0, st, B, D, W, T, out);
  return hipGetLastError();
}

}  // namespace IE_RNS

#if !defined(IE_RESOLVE_WIDE)
// The unescape command on a views batch (py:1660-1667): the fused resolve on the tiles, then the
// strings it deferred: unescaped into the pool and resolved as a deferred subset (results written
// at their places in the batch, bytes claimed from the same cursor). Asynchronous.
hipError_t launch_unescape_cmd(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                               uint64_t* sub_off, uint32_t* sub_len, uint32_t* sub_tid, hipStream_t st) {
  Work W0 = W;  // (the fused pass's emit: neither the telemetry nor the pool word, the call goes on)
  W0.stat_out = nullptr;
  W0.pool_out = nullptr;
  hipError_t e = IE_RNS::launch_resolve_impl(B, W0, T, out, cap, st, true);
  if (e != hipSuccess) return e;
  // the windowed-tile list is the deferred resolve's again
  e = hipMemsetAsync(W.defer_count, 0, sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  const uint64_t blocks = (B.n + kRBlock - 1) / kRBlock;
  hipLaunchKernelGGL(IE_RNS::k_unesc_deferred, dim3((uint32_t)(blocks < 1024 ? blocks : 1024)), dim3(kRBlock), 0, st, B,
                     W, sub_off, sub_len, sub_tid);
  Batch D{W.pool, sub_off, B.n, B.out_off, B.status, B.value_id, sub_tid, sub_len, B.out_len, W.udefer_list, W.udefer_count};
  return IE_RNS::launch_resolve_impl(D, W, T, out, cap, st, false);
}
#endif

#if !defined(IE_RESOLVE_WIDE)
// host-built patches of a device table (ie_table_set_update, ie_table_set_clock): one lane per patch
// of <= 256 bytes (whole 64-byte entries as four 16-byte moves)
__global__ void k_patch(const uint8_t* src, const uint64_t* dst, const uint32_t* soff, const uint32_t* len, uint32_t n) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint8_t* d = (uint8_t*)(uintptr_t)dst[k];
  const uint8_t* s = src + soff[k];
  const uint32_t l = len[k];
  if (l == sizeof(Entry) && ((uintptr_t)d & 15u) == 0) {
    for (uint32_t j = 0; j < sizeof(Entry) / 16; j++) gst4((uint4*)d + j, gld4((const uint4*)s + j));
    return;
  }
  for (uint32_t j = 0; j < l; j++) d[j] = s[j];
}

hipError_t launch_patch(const uint8_t* src, const uint64_t* dst, const uint32_t* soff, const uint32_t* len, uint32_t n,
                        hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_patch, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, soff, len, n);
  return hipGetLastError();
}

__global__ void k_patch_inline(const PatchInline a) {
  const uint32_t c = threadIdx.x;
  if (c >= a.n) return;
  const uint32_t w[4] = {a.data[c][0], a.data[c][1], a.data[c][2], a.data[c][3]}, l = a.len[c];
  uint8_t* d = (uint8_t*)(uintptr_t)a.dst[c];
  if (l == 16 && ((uintptr_t)d & 15u) == 0) {
    gst4((uint4*)d, make_uint4(w[0], w[1], w[2], w[3]));
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < 16; j++)
    if (j < l) d[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
}

hipError_t launch_patch_inline(const PatchInline& a, hipStream_t st) {
  if (!a.n || a.n > kPatchInlineN) return a.n ? hipErrorInvalidValue : hipSuccess;
  hipLaunchKernelGGL(k_patch_inline, dim3(1), dim3(kPatchInlineN), 0, st, a);
  return hipGetLastError();
}

// k_resolve on a views batch in two passes (IE_OPT_DEFER): the strings the chain jobs could not
// finish are listed by the first (the LEAN instances) and resolved by the second (the full ones) as
// a subset
hipError_t launch_resolve_deferring(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                                    uint64_t* sub_off, uint32_t* sub_len, uint32_t* sub_tid, hipStream_t st) {
  if (!B.out_len || !B.n) return hipErrorInvalidValue;
  // first pass: the LEAN instances (no exact evaluator, no literal path), which also write the
  // deferred strings' views (sub_off / sub_len / sub_tid) for the second pass
  const bool multi = B.table_id != nullptr;
  Work W1 = W;
  W1.defer_slow = 1;
  W1.sub_off = sub_off;
  W1.sub_len = sub_len;
  W1.sub_tid = multi ? sub_tid : nullptr;
  hipError_t e = IE_RNS::launch_resolve_impl(B, W1, T, out, cap, st, false, true, false, false);
  if (e != hipSuccess) return e;
  // the second pass appends its windowed tiles to the first's list (flagged as the subset's), and
  // ONE k_emit_windows writes both passes' windows, the total and the telemetry
  Work W2 = W;
  W2.defer_slow = 0;
  const Batch D{B.bytes, sub_off, B.n, B.out_off, B.status, B.value_id, multi ? sub_tid : nullptr, sub_len, B.out_len,
                W.udefer_list, W.udefer_count};
  e = IE_RNS::launch_resolve_impl(D, W2, T, out, cap, st, false, false, false, false);
  if (e != hipSuccess) return e;
  return IE_RNS::launch_emit(B, D, W, T, out, st);
}
#endif

#if defined(IE_RESOLVE_WIDE)
hipError_t launch_resolve512(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                             hipStream_t st) {
  return IE_RNS::launch_resolve_impl(B, W, T, out, cap, st);
}
#else
hipError_t launch_resolve(const Batch& B, const Work& W, const DevTable& T, uint8_t* out, uint64_t cap,
                          hipStream_t st, bool no_emit) {
  return IE_RNS::launch_resolve_impl(B, W, T, out, cap, st, false, false, no_emit);
}
hipError_t launch_debug_probe(const DevTable& T, const uint8_t* key, uint32_t klen, uint64_t* out, hipStream_t st) {
  return IE_RNS::launch_debug_probe_impl(T, key, klen, out, st);
}
bool kernels_cuckoo() {
#ifdef IE_CUCKOO
  return true;
#else
  return false;
#endif
}
#endif

}  // namespace ie
