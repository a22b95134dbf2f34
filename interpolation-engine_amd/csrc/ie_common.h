// ie_common.h — types shared by the host table builder and the gfx950 kernels.
//
// Device data layout of one inserts table (built once per get_interpdata snapshot, read-only):
//   pilots[nb]      uint16 per pilot group (about 4 keys per group): the displacement that sends
//                   every key of the group to its own entry (a perfect hash: each key has exactly
//                   ONE candidate entry). A lookup is two dependent reads, the pilot (L2-resident:
//                   50 KB for 100k keys) and then the entry
//   entries[m]      Entry (64 B): lengths, flags, arena offset, inline copies of the key (<= 16 B)
//                   and splice text (<= 28 B), value id; a lookup reads the first 48 bytes (the
//                   first 16 text bytes are all an inner nesting level needs); m ~ 1.25 * keys
//   arena[...]      every splice text (4-byte aligned) followed by its key (4-byte aligned)
// Lookup of key k in table t of the set: h = hash_key(k, seed, t); group g = ph_group(h, nb);
// slot = ph_slot(h, pilots[g]); the key is present iff entries[slot] holds it for table t (full
// byte compare and table index compare: exact, never a hash test).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define IE_HD __host__ __device__ __forceinline__
#else
#define IE_HD inline
#endif

namespace ie {

// Key hash: two 32-bit multiplicative lanes over the key's little-endian 4-byte words (zero
// padded), seeded with the table seed and the length; the high lane picks the pilot group
// (its top bits), the low lane the slot under the pilot (ph_slot mixes it). One multiply per
// word and lane (the device hashes keys straight from registers).
IE_HD uint64_t hash_word(uint64_t h, uint32_t w) {
  const uint32_t a = ((uint32_t)(h >> 32) ^ w) * 0x9E3779B1u;
  const uint32_t b = ((uint32_t)h ^ w) * 0xCC9E2D51u;
  return ((uint64_t)a << 32) | b;
}

// start of a key's hash: the table seed, the key length and the index of the table the key belongs
// to in a table set (0 for a single table), so one device table can hold many inserts dicts
IE_HD uint64_t hash_init(uint32_t n, uint64_t seed, uint32_t tid) {
  // the table index enters both lanes: equal keys of different tables must differ in the high
  // lane (their pilot group) and in the low lane (their slot under a shared pilot)
  return seed ^ (((uint64_t)(n ^ (tid << 11)) << 32) | (uint64_t)((n * 0x85EBCA77u) ^ tid));
}

// hash of n key bytes (any address space via the byte reader)
template <class ByteAt>
IE_HD uint64_t hash_key(uint32_t n, ByteAt at, uint64_t seed, uint32_t tid) {
  uint64_t h = hash_init(n, seed, tid);
  for (uint32_t j = 0; j < n; j += 4) {
    uint32_t w = 0;
    for (uint32_t b = 0; b < 4 && j + b < n; b++) w |= (uint32_t)at(j + b) << (8 * b);
    h = hash_word(h, w);
  }
  return h;
}

IE_HD uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

// Two-choice (cuckoo) placement, the one-trip table experiment (IE_CUCKOO builds; host env
// IE_CUCKOO=1): a key sits in one of its two candidate entries, both read in the same round.
IE_HD void ck_slots(uint64_t h, uint32_t m, uint32_t& s1, uint32_t& s2) {
  s1 = (uint32_t)(((uint64_t)fmix32((uint32_t)h) * m) >> 32);
  s2 = (uint32_t)(((uint64_t)fmix32((uint32_t)(h >> 32) ^ 0x5BD1E995u) * m) >> 32);
  if (s2 == s1) s2 = s1 + 1 == m ? 0u : s1 + 1;
}

// pilot group of a key hash (multiply-shift range reduction of the high word)
IE_HD uint32_t ph_group(uint64_t h, uint32_t nb) {
  return (uint32_t)(((uint64_t)(uint32_t)(h >> 32) * (uint64_t)nb) >> 32);
}
// entry slot of a key hash under its group's pilot (multiply-shift range reduction to [0, m))
IE_HD uint32_t ph_slot(uint64_t h, uint32_t pilot, uint32_t m) {
  return (uint32_t)(((uint64_t)fmix32((uint32_t)h ^ (pilot * 0x9E3779B9u)) * m) >> 32);
}


// get_simple_insertkey (py:477-495 / interp.rs:11-29) on n bytes of UTF-8 (any address space via
// the byte reader): true when the reference returns a truthy key (py) / Some (rs); koff / klen
// locate the key, content[1:-1] in characters. The py loop runs over characters with NO test that
// the edges are braces: 'a}b{c' is simple (key '}b{', the depth dips below 0 and comes back at the
// last character), so the edge test is "first or last character", not "first or last byte". The
// rs version requires a '{' first and a '}' last (interp.rs:14-16) and gives Some("") for "{}".
template <class ByteAt>
IE_HD bool simple_insertkey(ByteAt at, uint64_t n, uint32_t dialect, uint64_t& koff, uint64_t& klen) {
  koff = klen = 0;
  uint64_t nch = 0, l0 = n, last = 0;  // characters, bytes of the first, start of the last
  for (uint64_t k = 0; k < n; k++) {
    if ((at(k) & 0xC0u) == 0x80u) continue;  // a continuation byte: the same character
    if (nch == 1) l0 = k;
    last = k;
    nch++;
  }
  if (dialect == 1u && (nch < 2 || at(0) != '{' || at(n - 1) != '}')) return false;
  int64_t depth = 0;
  uint64_t ci = 0;
  for (uint64_t k = 0; k < n; k++) {
    const uint8_t c = at(k);
    if ((c & 0xC0u) == 0x80u) continue;
    if (c == '}') depth--;
    if ((depth == 0) != (ci == 0 || ci == nch - 1)) return false;
    if (c == '{') depth++;
    ci++;
  }
  if (nch <= 2) return dialect == 1u && nch == 2;  // py: '' is falsy; rs: Some("") for "{}"
  koff = l0;
  klen = last - l0;
  return true;
}

// Entry.flags
enum : uint32_t {
  EF_KIND_MASK = 7u,
  EF_SPLICE_OK = 1u << 3,      // the dialect's splice type rule passes (py:530 / interp.rs:71-80)
  EF_INERT = 1u << 4,          // splice text cannot alter brace/escape/placeholder structure
  EF_KEY_STR = 1u << 5,        // raw value usable as a lookup key (py: str only; rs: value_to_string)
  EF_KEY_UNHASHABLE = 1u << 6, // py: list/dict raw value as a dict key raises TypeError
  EF_OCCUPIED = 1u << 7,       // the entry holds a key
  EF_RAWALT = 1u << 8,         // splice text pre-resolved at build; the raw value sits before it
                               // in the arena as [raw text, 4-aligned][u32 raw length][text]
};
// bits 12-31 of Entry.flags: the index of the entry's table within its table set
constexpr uint32_t kTidShift = 12;
constexpr uint32_t kMaxTables = 1u << (32 - kTidShift);

// DevTable.flags
enum : uint32_t {
  TF_HAS_DIR = 1u,
  TF_LONG_KEYS = 2u,  // some key is 17-32 bytes long: k_resolve's chain jobs compare key tails (LK)
  TF_CUCKOO = 4u,     // two-choice placement (the IE_CUCKOO experiment), no pilots
};

constexpr uint32_t kInlineKey = 16;   // bytes of key kept inline in an entry
constexpr uint32_t kInlineText = 28;  // bytes of splice text kept inline in an entry

struct Entry {
  uint32_t key_len, text_len, flags, text_off;  // 16-byte word 0
  uint8_t key[kInlineKey];                      // word 1: zero padded
  uint8_t text[kInlineText];                    // words 2, 3.xyz: zero padded (a <= 16 B text is word 2)
  uint32_t vid;                                 // word 3.w
};
static_assert(sizeof(Entry) == 64, "Entry must stay one 64-byte block");

// the key's arena offset: right after the (4-aligned) splice text
IE_HD uint32_t key_off_of(uint32_t text_off, uint32_t text_len) { return text_off + ((text_len + 3u) & ~3u); }

struct DevTable {
  const Entry* entries;
  const uint16_t* pilots;
  const uint8_t* arena;
  uint64_t seed;
  uint32_t m;     // entries
  uint32_t nb;    // pilot groups
  uint32_t n_entries;
  uint32_t n_tables;  // inserts dicts in the set (strings pick one with Batch.table_id)
  uint32_t dialect;
  uint32_t flags;
  uint64_t maxtext;
};

// internal status: routed to the literal (complex) kernel
constexpr uint8_t kStatusPending = 0xFE;
// internal status: left to the fused unescape command's deferred pass (rewritten by it)
constexpr uint8_t kStatusDeferred = 0xFD;

// ------------------------------------------------------------------------------------------
// Synthetic workloads: counter-based splitmix64, identical on host and device.
// ------------------------------------------------------------------------------------------
IE_HD uint64_t splitmix(uint64_t& s) {
  s += 0x9E3779B97F4A7C15ull;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct SynthParams {
  int32_t config;     // 2, 3 or 4
  uint64_t seed;
  uint32_t n_keys;    // config 2: k0..k{n_keys-1}
  uint32_t n_q;       // config 3/4: q-0..q-{n_q-1}
  uint32_t n_i;       // config 3/4: i0..i{n_i-1}
  uint32_t n_chain;   // config 4: c-0..c-{n_chain-1} (brace-bearing values)
};

// filler alphabet: ASCII [a-z0-9 .,:;-] plus 5% multibyte code points (é, €, 😀);
// never '{', '}', '\\' or U+3020.
IE_HD uint32_t synth_filler(uint64_t& st, uint8_t* out, uint32_t nbytes) {
  const char* ascii = "abcdefghijklmnopqrstuvwxyz0123456789 .,:;-";
  uint32_t w = 0;
  while (w < nbytes) {
    uint64_t r = splitmix(st);
    uint32_t left = nbytes - w;
    if ((r % 100) < 5 && left >= 2) {
      uint32_t pick = (uint32_t)((r >> 8) % 3);
      if (pick == 2 && left >= 4) {
        if (out) { out[w] = 0xF0; out[w + 1] = 0x9F; out[w + 2] = 0x98; out[w + 3] = 0x80; }
        w += 4;
        continue;
      }
      if (pick >= 1 && left >= 3) {
        if (out) { out[w] = 0xE2; out[w + 1] = 0x82; out[w + 2] = 0xAC; }
        w += 3;
        continue;
      }
      if (out) { out[w] = 0xC3; out[w + 1] = 0xA9; }
      w += 2;
      continue;
    }
    if (out) out[w] = (uint8_t)ascii[(r >> 16) % 42];
    w += 1;
  }
  return w;
}

IE_HD uint32_t put_dec(uint8_t* out, uint32_t v) {
  uint8_t tmp[12];
  uint32_t n = 0;
  do {
    tmp[n++] = (uint8_t)('0' + v % 10);
    v /= 10;
  } while (v);
  for (uint32_t k = 0; k < n; k++)
    if (out) out[k] = tmp[n - 1 - k];
  return n;
}

IE_HD uint64_t synth_state(const SynthParams& P, uint64_t i) {
  uint64_t s = P.seed ^ ((uint64_t)P.config << 56);
  s += (i + 1) * 0xD1B54A32D192ED03ull;
  splitmix(s);
  return s;
}

// Byte length of synthetic string i (the first draw of its stream).
IE_HD uint32_t synth_len(const SynthParams& P, uint64_t i) {
  uint64_t st = synth_state(P, i);
  return 48u + (uint32_t)(splitmix(st) % 33u);
}

// Writes string i (exactly synth_len bytes) to out.
IE_HD uint32_t synth_string(const SynthParams& P, uint64_t i, uint8_t* out) {
  uint64_t st = synth_state(P, i);
  const uint32_t L = 48u + (uint32_t)(splitmix(st) % 33u);
  // references
  uint8_t ref[4][40];
  uint32_t rlen[4];
  uint32_t R;
  if (P.config == 2) {
    R = 1 + (uint32_t)(splitmix(st) % 3);
    for (uint32_t r = 0; r < R; r++) {
      uint32_t j = (uint32_t)(splitmix(st) % P.n_keys);
      uint32_t w = 0;
      ref[r][w++] = '{';
      ref[r][w++] = 'k';
      w += put_dec(ref[r] + w, j);
      ref[r][w++] = '}';
      rlen[r] = w;
    }
  } else if (P.config == 3) {
    R = 1 + (uint32_t)(splitmix(st) % 2);
    for (uint32_t r = 0; r < R; r++) {
      uint32_t m = (uint32_t)(splitmix(st) % P.n_i);
      uint32_t w = 0;
      ref[r][w++] = '{';
      ref[r][w++] = 'q';
      ref[r][w++] = '-';
      ref[r][w++] = '{';
      ref[r][w++] = 'i';
      w += put_dec(ref[r] + w, m);
      ref[r][w++] = '}';
      ref[r][w++] = '}';
      rlen[r] = w;
    }
  } else {
    // config 4: 1-2 chain refs of depth 1/2/3/4 = 40/30/20/10 %:
    //   {q-N}  {q-{iM}}  {q-{a-{iM}}}  {q-{a-{b-{iM}}}}
    // per string: 2 % replace ref 0 by {c-N} (a brace-bearing value: re-resolved, the complex
    // path), 1 % by a missing key {zz-N} (status row); 10 % add an escaped \{lit\} segment.
    R = 1 + (uint32_t)(splitmix(st) % 2);
    for (uint32_t r = 0; r < R; r++) {
      const uint32_t u = (uint32_t)(splitmix(st) % 100);
      const uint32_t depth = u < 40 ? 1 : u < 70 ? 2 : u < 90 ? 3 : 4;
      uint32_t w = 0;
      ref[r][w++] = '{';
      ref[r][w++] = 'q';
      ref[r][w++] = '-';
      if (depth == 1) {
        w += put_dec(ref[r] + w, (uint32_t)(splitmix(st) % P.n_q));
      } else {
        if (depth >= 3) { ref[r][w++] = '{'; ref[r][w++] = 'a'; ref[r][w++] = '-'; }
        if (depth == 4) { ref[r][w++] = '{'; ref[r][w++] = 'b'; ref[r][w++] = '-'; }
        ref[r][w++] = '{';
        ref[r][w++] = 'i';
        w += put_dec(ref[r] + w, (uint32_t)(splitmix(st) % P.n_i));
        for (uint32_t k = 1; k < depth; k++) ref[r][w++] = '}';
      }
      ref[r][w++] = '}';
      rlen[r] = w;
    }
    const uint32_t u = (uint32_t)(splitmix(st) % 100);
    if (u < 3) {
      uint32_t w = 0;
      ref[0][w++] = '{';
      if (u < 2) {
        ref[0][w++] = 'c';
        ref[0][w++] = '-';
        w += put_dec(ref[0] + w, (uint32_t)(splitmix(st) % P.n_chain));
      } else {
        ref[0][w++] = 'z';
        ref[0][w++] = 'z';
        ref[0][w++] = '-';
        w += put_dec(ref[0] + w, (uint32_t)(splitmix(st) % 1000));
      }
      ref[0][w++] = '}';
      rlen[0] = w;
    }
    if ((uint32_t)(splitmix(st) % 100) < 10) {
      const char* lit = "\\{lit\\}";
      for (uint32_t k = 0; k < 7; k++) ref[R][k] = (uint8_t)lit[k];
      rlen[R] = 7;
      R++;
    }
  }
  uint32_t refbytes = 0;
  for (uint32_t r = 0; r < R; r++) refbytes += rlen[r];
  uint32_t F = L > refbytes + 1 ? L - refbytes : 1;  // L >= 48 > refbytes always
  // split F filler bytes into R+1 gaps, gap 0 >= 1 (no whole-string simple refs)
  uint32_t gap[5];
  uint32_t rest = F - 1;
  for (uint32_t g = 0; g < R; g++) {
    uint32_t take = rest ? (uint32_t)(splitmix(st) % (rest + 1)) : 0;
    gap[g] = take;
    rest -= take;
  }
  gap[R] = rest;
  gap[0] += 1;
  uint32_t w = 0;
  for (uint32_t g = 0; g <= R; g++) {
    w += synth_filler(st, out ? out + w : nullptr, gap[g]);
    if (g < R) {
      for (uint32_t k = 0; k < rlen[g]; k++)
        if (out) out[w + k] = ref[g][k];
      w += rlen[g];
    }
  }
  return w;  // == L
}

}  // namespace ie
