// ie_wildcard.hip — k_wildcard: wildcard match / capture over a packed batch of strings
// (is_wildcard_match / get_wildcard_matches, py:553-567; rust-project/src/runtime.rs:1633-1647,
// 1754-1775), the matcher behind goto_map / replace_map / delete_except (py:1688-1773).
//
// The reference builds the regex '^' + re.escape(w.replace('*', '〠')).replace('〠', '(.*)') + '$'
// (DOTALL) and runs re.match / re.findall. So a pattern is literals L0 (.*) L1 ... (.*) Lk, split
// at every '*' and every U+3020 (a literal U+3020 in the wildcard becomes a group too), and:
//   * the match is anchored at 0 and ends at n, or at n-1 when the string ends in '\n' ('$'
//     also matches before a trailing newline);
//   * backtracking tries the groups longest-first, left to right, so the captures are the
//     lexicographically largest (g1, ..., gk): every literal at its RIGHTMOST feasible position,
//     found right to left (Lk fixed by the end, then each L_j the last occurrence that ends before
//     L_{j+1} starts), and the end n is preferred over n-1 (it is never lexicographically
//     smaller);
//   * a pattern without groups "captures" its whole match (re.findall returns the match), i.e.
//     L0 without the trailing newline.
// Byte positions equal the regex's code-point positions: a valid UTF-8 literal can only match at
// code-point boundaries, and every other position is fixed by the literals and the end.
//
// IE_DIALECT_RS (runtime.rs:1633-1647, 1754-1775, the regex crate): only '*' is a group, '$'
// matches at the end only, and a group-less wildcard captures nothing.
//
// One wave per string (wave-uniform control flow, byte comparisons spread over the 64 lanes);
// strings up to kWcStage bytes are staged in LDS, longer ones are read from global memory.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ie_device.h"
#include "ie_kernels.h"

namespace ie {

constexpr uint32_t kWcStage = 2048;  // bytes per wave staged in LDS
constexpr uint32_t kWcWaves = 4;

typedef __attribute__((address_space(3))) uint8_t wc_lds_u8;

struct WcStr {
  const uint8_t* g;   // global copy
  const wc_lds_u8* l; // LDS copy (staged) or null
  __device__ __forceinline__ uint8_t operator[](uint32_t i) const { return l ? l[i] : gld(g + i); }
};

// s[at .. at + len) == lit (wave-uniform arguments; every lane compares a strided part)
__device__ __forceinline__ bool wc_eq(const WcStr& s, uint32_t at, const uint8_t* lit, uint32_t len) {
  bool ok = true;
  for (uint32_t b = lane_id(); b < len; b += 64) ok &= s[at + b] == gld(lit + b);
  return __ballot(!ok) == 0;
}

// the rightmost q in [lo, hi - len] with s[q .. q + len) == lit, or -1 (wave-uniform)
__device__ int64_t wc_rfind(const WcStr& s, uint32_t lo, uint32_t hi, const uint8_t* lit, uint32_t len) {
  if (hi < lo + len) return -1;
  const uint32_t lane = lane_id();
  const uint8_t first = len ? gld(lit) : 0;
  for (int64_t top = (int64_t)(hi - len); top >= (int64_t)lo; top -= 64) {
    const int64_t q = top - (int64_t)lane;
    bool m = q >= (int64_t)lo;
    if (m && len) m = s[(uint32_t)q] == first;
    for (uint32_t b = 1; __any(m) && b < len; b++) m = m && s[(uint32_t)q + b] == gld(lit + b);
    const uint64_t bal = __ballot(m);
    if (bal) return top - (int64_t)__builtin_ctzll(bal);
  }
  return -1;
}

// Per string i: the first pattern p of [lo_i, hi_i) (all patterns when range is null) that
// matches, or -1; its captures as {start, length} byte pairs (caps + i * 2 * kWcMaxCap) and their
// count (ncap[i]).
__global__ __launch_bounds__(64 * kWcWaves) void k_wildcard(WcSet P, const uint8_t* bytes, const uint64_t* off, uint64_t n,
                                                            const uint32_t* range, int32_t* match, uint8_t* ncap,
                                                            uint32_t* caps) {
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[kWcWaves][kWcStage];
  __shared__ uint32_t s_pos[kWcWaves][kWcMaxCap + 1];
  const uint32_t wave = threadIdx.x >> 6, lane = lane_id();
  const uint64_t waves = (uint64_t)gridDim.x * kWcWaves;
  for (uint64_t i = (uint64_t)blockIdx.x * kWcWaves + wave; i < n; i += waves) {
    const uint64_t so = off[i];
    const uint32_t len = (uint32_t)(off[i + 1] - so);
    WcStr s{bytes + so, nullptr};
    if (len <= kWcStage) {
      wc_lds_u8* st = (wc_lds_u8*)s_stage[wave];
      for (uint32_t k = lane; k < len; k += 64) st[k] = gld(bytes + so + k);
      __builtin_amdgcn_wave_barrier();
      s.l = st;
    }
    uint32_t lo = 0, hi = P.n_pat;
    if (range) {
      lo = range[2 * i];
      hi = range[2 * i + 1];
      hi = hi < P.n_pat ? hi : P.n_pat;
    }
    int32_t found = -1;
    uint32_t k_found = 0;
    uint32_t* pos = s_pos[wave];  // literal start positions of the match (pos[j] for L_j)
    for (uint32_t p = lo; p < hi && found < 0; p++) {
      const uint32_t l0 = P.pat_lit[p], nl = P.pat_lit[p + 1] - l0, k = nl - 1;
      const uint32_t len0 = P.lit_len[l0];
      if (len0 > len || !wc_eq(s, 0, P.bytes + P.lit_off[l0], len0)) continue;
      const bool nl_end = !P.rs && len > 0 && s[len - 1] == '\n';  // py '$'; the regex crate's is the end only
      if (k == 0) {
        if (len0 == len || (nl_end && len0 + 1 == len)) {
          found = (int32_t)p;
          k_found = 0;
        }
        continue;
      }
      // the end n first, then n - 1 before a trailing newline
      for (int e = 0; e < 2 && found < 0; e++) {
        if (e == 1 && !nl_end) break;
        const uint32_t E = len - (uint32_t)e;
        const uint32_t lk = P.lit_len[l0 + k];
        if (E < len0 + lk) continue;
        uint32_t R = E - lk;
        if (!wc_eq(s, R, P.bytes + P.lit_off[l0 + k], lk)) continue;
        if (lane == 0) pos[k] = R;
        bool ok = true;
        for (uint32_t j = k - 1; j >= 1 && ok; j--) {
          const int64_t q = wc_rfind(s, len0, R, P.bytes + P.lit_off[l0 + j], P.lit_len[l0 + j]);
          ok = q >= 0;
          if (ok) {
            R = (uint32_t)q;
            if (lane == 0) pos[j] = R;
          }
        }
        if (ok) {
          found = (int32_t)p;
          k_found = k;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) match[i] = found;
    uint32_t* c = caps + i * 2 * kWcMaxCap;
    if (found < 0) {
      if (lane == 0) ncap[i] = 0;
      continue;
    }
    const uint32_t l0 = P.pat_lit[found];
    if (k_found == 0) {  // no group: re.findall returns the whole match (py); no capture (rs)
      if (lane == 0) {
        ncap[i] = P.rs ? 0 : 1;
        c[0] = 0;
        c[1] = P.lit_len[l0];
      }
      continue;
    }
    if (lane == 0) ncap[i] = (uint8_t)k_found;
    if (lane < k_found) {  // group j = lane + 1 runs from the end of L_j-1 to the start of L_j
      const uint32_t j = lane + 1;
      const uint32_t start = j == 1 ? P.lit_len[l0] : pos[j - 1] + P.lit_len[l0 + j - 1];
      c[2 * lane] = start;
      c[2 * lane + 1] = pos[j] - start;
    }
  }
}

hipError_t launch_wildcard(const WcSet& P, const uint8_t* bytes, const uint64_t* off, uint64_t n,
                           const uint32_t* range, int32_t* match, uint8_t* ncap, uint32_t* caps, hipStream_t st) {
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + kWcWaves - 1) / kWcWaves;
  const uint32_t grid = (uint32_t)(blocks < 8192 ? blocks : 8192);
  hipLaunchKernelGGL(k_wildcard, dim3(grid), dim3(64 * kWcWaves), 0, st, P, bytes, off, n, range, match, ncap, caps);
  return hipGetLastError();
}

}  // namespace ie
