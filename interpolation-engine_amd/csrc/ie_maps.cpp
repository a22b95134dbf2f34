// ie_maps.cpp — the map commands of the reference's interpreter over the states of a table set
// (SURVEY §8f-2): goto_map (py:1689-1711), replace_map's replace_str (py:1713-1745) and delete /
// delete_except (py:1843-1868); rust-project/src/runtime.rs:1085-1169, 1649-1731, 1754-1775.
//
// State s is table s of the set. Every interpolation runs in k_resolve (run_host) and every
// wildcard test in k_wildcard (ie_wildcard_match_batch): a command over any number of states is a
// handful of device batches. The host code here is the commands' control flow: which strings go
// into the next batch, the first matching map, the order in which the reference raises, and
// repeat_until_done's fixed point.
//
// replace_map interpolates a matched map's value against `inserts | extra_inserts`, the captures
// bound to '1', '2', ... (py:1732-1738). When the captures are inert (no unescaped brace, no
// U+3020, no escape hazard at their edges: the table builder's EF_INERT rule) and the value is
// properly nested with no U+3020, that equals interpolating the value with each `{N}` pair of a
// capture index replaced by the capture against the state's own table: for properly nested strings
// with inert spliced values the reference's rightmost-innermost loop is a left-to-right stack
// evaluation, in which a `{N}` pair resolves to its capture before anything reads it,
// and an inert capture cannot change what the loop sees around it. Any other value resolves
// against a table of its own: the state's entries (from the table's host mirror) and the captures.
#include <stdlib.h>

#include <algorithm>
#include <deque>
#include <unordered_map>

#include "ie_internal.h"

namespace {

constexpr uint32_t kMaxPasses = 100000;  // repeat_until_done without a fixed point: IE_DIVERGED


struct MapOut {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off{0};
  std::vector<uint8_t> status;
  std::vector<uint32_t> where, vid;
  std::vector<int32_t> chosen;
  void push(std::string_view s, uint8_t st, uint32_t w, int32_t c, uint32_t v = IE_VID_NONE) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    off.push_back(bytes.size());
    status.push_back(st);
    where.push_back(w);
    chosen.push_back(c);
    vid.push_back(v);
  }
};

int emit(MapOut& m, ie_map_result** out) {
  ie_map_result* r = new ie_map_result{};
  const uint64_t n = m.status.size();
  r->n = n;
  r->bytes_len = m.bytes.size();
  r->bytes = new uint8_t[m.bytes.size() + 1];
  if (!m.bytes.empty()) memcpy(r->bytes, m.bytes.data(), m.bytes.size());
  r->offsets = new uint64_t[n + 1];
  memcpy(r->offsets, m.off.data(), (n + 1) * sizeof(uint64_t));
  r->status = new uint8_t[n + 1];
  r->where = new uint32_t[n + 1];
  r->chosen = new int32_t[n + 1];
  r->value_id = new uint32_t[n + 1];
  for (uint64_t i = 0; i < n; i++) {
    r->status[i] = m.status[i];
    r->where[i] = m.where[i];
    r->chosen[i] = m.chosen[i];
    r->value_id[i] = m.vid[i];
  }
  *out = r;
  return IE_SUCCESS;
}

// strings for one device batch: packed, one table (state) id each
struct Strs {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> off{0};
  std::vector<uint32_t> tid;
  void add(std::string_view s, uint32_t t) {
    bytes.insert(bytes.end(), s.begin(), s.end());
    off.push_back(bytes.size());
    tid.push_back(t);
  }
  uint64_t size() const { return tid.size(); }
  void reserve(uint64_t n, uint64_t nbytes) {  // (no regrowth copies of a batch of KB-long texts)
    bytes.reserve(nbytes);
    off.reserve(n + 1);
    tid.reserve(n);
  }
};

// the results of a batch: str() of each (py:1692, 1698-1699, 1722, 1738: a whole-string key's
// typed result is str()-ed), the status (IE_OK_VALUE kept, with its value id)
struct Res {
  std::vector<std::string_view> text;  // into the batch's bytes, or into `owned` (a typed result's str())
  std::vector<uint8_t> st;
  std::vector<uint32_t> vid;
  std::deque<std::string> owned;
  ie_batch* b = nullptr;
  Res() = default;
  Res(const Res&) = delete;
  Res& operator=(const Res&) = delete;
  ~Res() { ie_batch_free(b); }
};

// str() of the raw insert behind a whole-string result (py:510-514): the entry's rendering (the
// raw text of a pre-resolved one), or the clock's text for the clock ids
ie_clock table_clock(const ie_table* t);

// the slot holding value id vid (table tb, or any table when tb is UINT32_MAX), UINT32_MAX: none
uint32_t slot_of_vid(const ie_table* t, uint32_t vid, uint32_t tb = UINT32_MAX) {
  std::lock_guard<std::mutex> lock(t->vid_mu);  // (concurrent readers of one table)
  if (!t->vid_ok) {
    t->vid_slot.assign(t->next_vid, UINT32_MAX);
    for (uint32_t s = 0; s < (uint32_t)t->h_entries.size(); s++) {
      const Entry& e = t->h_entries[s];
      if (!(e.flags & EF_OCCUPIED) || e.vid >= IE_VID_CLOCK_HHMMSS) continue;
      if (e.vid >= t->vid_slot.size()) t->vid_slot.resize(e.vid + 1, UINT32_MAX);
      t->vid_slot[e.vid] = s;
    }
    t->vid_ok = true;
  }
  auto holds = [&](uint32_t s) {
    const Entry& e = t->h_entries[s];
    return (e.flags & EF_OCCUPIED) && e.vid == vid && (tb == UINT32_MAX || (e.flags >> kTidShift) == tb);
  };
  uint32_t s = vid < t->vid_slot.size() ? t->vid_slot[vid] : UINT32_MAX;
  if (s == UINT32_MAX || !holds(s)) {  // (a caller's ids shared between tables: the slow way)
    s = UINT32_MAX;
    for (uint32_t k = 0; k < (uint32_t)t->h_entries.size() && s == UINT32_MAX; k++)
      if (holds(k)) s = k;
  }
  return s;
}

// an entry's stored text: the raw text of a pre-resolved one
std::string_view entry_text(const ie_table* t, const Entry& e) {
  const uint8_t* a = t->h_arena.data();
  if (e.flags & EF_RAWALT) {
    uint32_t rl;
    memcpy(&rl, a + e.text_off - 4, 4);
    return std::string_view((const char*)a + e.text_off - 4 - ((rl + 3u) & ~3u), rl);
  }
  return std::string_view((const char*)a + e.text_off, e.text_len);
}

bool value_str(const ie_table* t, uint32_t tb, uint32_t vid, std::string& out) {
  if (vid == IE_VID_CLOCK_HHMM || vid == IE_VID_CLOCK_HHMMSS) {  // (one clock for every table of a set)
    const ie_clock c = table_clock(t);
    char buf[16];
    snprintf(buf, sizeof buf, vid == IE_VID_CLOCK_HHMM ? "%02d:%02d" : "%02d:%02d:%02d", c.hour, c.minute, c.second);
    out = buf;
    return true;
  }
  const uint32_t s = slot_of_vid(t, vid, tb);
  if (s == UINT32_MAX) return false;
  out.assign(entry_text(t, t->h_entries[s]));
  return true;
}

int interp(ie_exec* x, const ie_table* t, const Strs& in, Res& r) {
  const uint64_t n = in.size();
  r.text.assign(n, std::string_view());
  r.st.assign(n, IE_OK_STR);
  r.vid.assign(n, IE_VID_NONE);
  if (!n) return IE_SUCCESS;
  ie_batch_free(r.b);
  r.b = nullptr;
  // A py string with no '{' and no U+3020 lead byte is its own interpolation (py:505-541: no
  // simple key, the loop never starts, the escapes' protection is undone): such strings (a map's
  // literal keys, a value's plain output going round repeat_until_done again) skip the device;
  // every other string goes to k_resolve.
  std::vector<uint64_t> dev;
  Strs sub;
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t* p = in.bytes.data() + in.off[i];
    const uint64_t len = in.off[i + 1] - in.off[i];
    if (t->dialect == IE_DIALECT_PY && !memchr(p, '{', len) && !memchr(p, 0xE3, len)) {
      r.text[i] = std::string_view((const char*)p, len);
      continue;
    }
    dev.push_back(i);
  }
  if (dev.empty()) return IE_SUCCESS;
  const bool all = dev.size() == n;
  if (!all)
    for (uint64_t i : dev)
      sub.add(std::string_view((const char*)in.bytes.data() + in.off[i], in.off[i + 1] - in.off[i]), in.tid[i]);
  const Strs& q = all ? in : sub;
  int rc = run_host(x, kOpInterp, t, q.bytes.data(), q.off.data(), q.size(), &r.b, q.tid.data());
  if (rc) return rc;
  const ie_batch* b = r.b;
  for (uint64_t k = 0; k < dev.size(); k++) {
    const uint64_t i = dev[k];
    r.st[i] = b->status[k];
    if (b->status[k] == IE_OK_STR) {
      r.text[i] = std::string_view((const char*)b->bytes + b->offsets[k], b->offsets[k + 1] - b->offsets[k]);
    } else if (b->status[k] == IE_OK_VALUE) {
      r.vid[i] = b->value_id[k];
      r.owned.emplace_back();
      if (!value_str(t, in.tid[i], b->value_id[k], r.owned.back()))
        return fail(IE_ERR_INVALID, "a typed result's value id is not in the table");
      r.text[i] = r.owned.back();
    }
  }
  return IE_SUCCESS;
}

inline bool ok(uint8_t st) { return st == IE_OK_STR || st == IE_OK_VALUE; }

// first-match of strings against per-string ranges of one wildcard list (k_wildcard)
struct Match {
  std::vector<int32_t> match;
  std::vector<uint8_t> ncap;
  std::vector<uint32_t> caps;
};
int match_first(ie_exec* x, const ie_table* t, const std::vector<std::string>& pats, const Strs& strs,
                const std::vector<uint32_t>& range, Match& m) {
  const uint64_t n = strs.size();
  m.match.assign(n, -1);
  m.ncap.assign(n, 0);
  m.caps.assign(n * 2 * IE_WC_MAX_CAP, 0);
  if (!n || pats.empty()) return IE_SUCCESS;
  std::vector<uint8_t> pb;
  std::vector<uint64_t> po{0};
  for (const std::string& p : pats) {
    pb.insert(pb.end(), p.begin(), p.end());
    po.push_back(pb.size());
  }
  // the exec's cache of compiled lists (the 64 most recent)
  std::string sig(1, (char)t->dialect);
  for (size_t k = 0; k < pats.size(); k++) sig += std::to_string(po[k + 1] - po[k]) + ":";
  sig.append((const char*)pb.data(), pb.size());
  ie_wildcards* w = nullptr;
  auto& cache = x->wc_cache;
  for (size_t k = 0; k < cache.size() && !w; k++) {
    if (cache[k].first != sig) continue;
    w = cache[k].second;
    std::rotate(cache.begin() + k, cache.begin() + k + 1, cache.end());  // (to the back: most recent)
  }
  Trace tr("match");
  if (!w) {
    tr.mark("wc lookup", cache.size());
    int rc = ie_wildcards_build(pb.data(), po.data(), (uint32_t)pats.size(), t->dialect, x->device, &w);
    if (rc) return rc;
    if (cache.size() >= 64) {
      ie_wildcards_free(cache.front().second);
      cache.erase(cache.begin());
    }
    cache.emplace_back(std::move(sig), w);
    tr.mark("wc build", pats.size());
  }
  const int rc = ie_wildcard_match_batch(x, w, strs.bytes.data(), strs.off.data(), n,
                                         range.empty() ? nullptr : range.data(), m.match.data(), m.ncap.data(),
                                         m.caps.data());
  tr.mark("wc batch", n);
  return rc;
}

// the pattern range of a key list in `pats`, appended once per distinct list (states whose map
// keys interpolate to the same texts share one block)
struct Blocks {
  std::vector<std::string> pats;
  std::unordered_multimap<uint64_t, std::pair<uint32_t, uint32_t>> seen;  // (hash of the list -> its block)
  std::pair<uint32_t, uint32_t> range(const std::vector<std::string>& keys, uint32_t upto) {
    uint64_t h = 0xcbf29ce484222325ull ^ upto;
    for (uint32_t j = 0; j < upto; j++) {
      for (const char c : keys[j]) h = (h ^ (uint8_t)c) * 0x100000001b3ull;
      h = (h ^ keys[j].size()) * 0x9E3779B97F4A7C15ull;
    }
    auto eq = seen.equal_range(h);
    for (auto it = eq.first; it != eq.second; ++it) {
      const auto rg = it->second;
      if (rg.second - rg.first != upto) continue;
      bool same = true;
      for (uint32_t j = 0; j < upto && same; j++) same = pats[rg.first + j] == keys[j];
      if (same) return rg;
    }
    const uint32_t lo = (uint32_t)pats.size();
    for (uint32_t j = 0; j < upto; j++) pats.push_back(keys[j]);
    const std::pair<uint32_t, uint32_t> rg{lo, (uint32_t)pats.size()};
    seen.emplace(h, rg);
    return rg;
  }
};

// may the captures be spliced into the value text before interpolating it (see the file header)?
bool substitutable(std::string_view v) {
  int64_t depth = 0;
  for (size_t i = 0; i < v.size(); i++) {
    const uint8_t c = (uint8_t)v[i];
    if (c == 0xE3 && i + 2 < v.size() && (uint8_t)v[i + 1] == 0x80 && (uint8_t)v[i + 2] == 0xA0) return false;
    const bool esc = i > 0 && v[i - 1] == '\\';  // py:505-508: '\{' / '\}' are text
    if (c == '{' && !esc) depth++;
    if (c == '}' && !esc && --depth < 0) return false;
  }
  return depth == 0;
}

// the value text with every unescaped `{N}` pair of a capture index replaced by that capture,
// appended to out (a batch's bytes: no intermediate string)
template <class Out>
void substitute(Out& out, std::string_view v, const std::vector<std::string_view>& caps) {
  size_t i = 0;
  while (i < v.size()) {
    if (v[i] == '{' && !(i > 0 && v[i - 1] == '\\')) {
      size_t j = i + 1;
      while (j < v.size() && v[j] >= '0' && v[j] <= '9') j++;
      if (j < v.size() && v[j] == '}' && j > i + 1 && v[i + 1] != '0' && j - i - 1 <= 6) {
        const uint64_t k = strtoull(std::string(v.substr(i + 1, j - i - 1)).c_str(), nullptr, 10);
        if (k >= 1 && k <= caps.size()) {
          out.insert(out.end(), caps[k - 1].begin(), caps[k - 1].end());
          i = j + 1;
          continue;
        }
      }
    }
    out.push_back((typename Out::value_type)v[i]);
    i++;
  }
}

// the clock a table was last given (its 'HH:MM:SS' entry)
ie_clock table_clock(const ie_table* t) {
  ie_clock c{0, 0, 0};
  for (uint32_t s : t->clock_slots) {
    if (s == UINT32_MAX) continue;
    const Entry& e = t->h_entries[s];
    if (e.vid == IE_VID_CLOCK_HHMMSS && e.text_len == 8) {
      const char* p = (const char*)t->h_arena.data() + e.text_off;
      c.hour = (p[0] - '0') * 10 + (p[1] - '0');
      c.minute = (p[3] - '0') * 10 + (p[4] - '0');
      c.second = (p[6] - '0') * 10 + (p[7] - '0');
      break;
    }
  }
  return c;
}

// a table set whose table h is state owner[h]'s dict (from the mirror: keys, raw texts, kinds) with
// extra[h] bound over it (`inserts | extra_inserts`, py:1734-1738)
int table_with(ie_exec* x, const ie_table* t, const std::vector<uint32_t>& owner,
               const std::vector<std::vector<std::pair<std::string, std::string>>>& extra, ie_table** out) {
  std::vector<std::vector<uint32_t>> slots(t->n_tables);
  std::vector<bool> want(t->n_tables, false);
  for (uint32_t o : owner) want[o] = true;
  for (uint32_t s = 0; s < (uint32_t)t->h_entries.size(); s++) {
    const Entry& e = t->h_entries[s];
    const uint32_t tb = e.flags >> kTidShift;
    if ((e.flags & EF_OCCUPIED) && e.vid < IE_VID_CLOCK_HHMMSS && want[tb]) slots[tb].push_back(s);
  }
  std::vector<std::string> texts;
  std::vector<ie_kv> kv;
  std::vector<uint64_t> start{0};
  texts.reserve(owner.size() * 4);
  // (texts first: the kv entries point into them)
  for (size_t h = 0; h < owner.size(); h++) {
    for (uint32_t s : slots[owner[h]]) {
      std::string v;
      value_str(t, owner[h], t->h_entries[s].vid, v);
      texts.push_back(std::move(v));
    }
  }
  size_t ti = 0;
  for (size_t h = 0; h < owner.size(); h++) {
    for (uint32_t s : slots[owner[h]]) {
      const Entry& e = t->h_entries[s];
      const std::string_view k = mirror_key(t, e);
      kv.push_back(ie_kv{k.data(), k.size(), texts[ti].data(), texts[ti].size(), (int32_t)(e.flags & EF_KIND_MASK), 0});
      ti++;
    }
    for (const auto& kvp : extra[h])  // (the last duplicate wins: the captures override the state)
      kv.push_back(ie_kv{kvp.first.data(), kvp.first.size(), kvp.second.data(), kvp.second.size(), IE_KIND_STR, 0});
    start.push_back(kv.size());
  }
  const ie_clock clk = table_clock(t);
  return ie_table_set_build(kv.data(), start.data(), (uint32_t)owner.size(), t->dialect, &clk,
                            (t->dev.flags & TF_HAS_DIR) ? IE_TABLE_HAS_INSERTS_DIR : 0u, x->device, out);
}

}  // namespace

extern "C" {

// the stored value behind a value id (any table of the set: the ids are unique in a set), from the
// host mirror: its kind and its text (a pre-resolved entry's raw text); valid until the next update
int ie_table_value(const ie_table* t, uint32_t vid, int32_t* kind, const char** text, uint64_t* len) {
  if (!t || !kind || !text || !len) return fail(IE_ERR_INVALID, "null argument");
  if (vid >= IE_VID_CLOCK_HHMMSS) return fail(IE_ERR_INVALID, "a clock id has no stored value");
  const uint32_t s = slot_of_vid(t, vid);
  if (s == UINT32_MAX) return fail(IE_ERR_INVALID, "value id not in the table");
  const Entry& e = t->h_entries[s];
  const std::string_view v = entry_text(t, e);
  *kind = (int32_t)(e.flags & EF_KIND_MASK);
  *text = v.data();
  *len = v.size();
  return IE_SUCCESS;
}

void ie_map_result_free(ie_map_result* r) {
  if (!r) return;
  delete[] r->bytes;
  delete[] r->offsets;
  delete[] r->status;
  delete[] r->where;
  delete[] r->chosen;
  delete[] r->value_id;
  delete r;
}

int ie_goto_map(ie_exec* x, const ie_table* t, const char* text, uint64_t text_len, const ie_map_pair* maps,
                uint32_t n_maps, ie_map_result** out) {
  if (!x || !t || !out || (text_len && !text) || (n_maps && !maps)) return fail(IE_ERR_INVALID, "null argument");
  *out = nullptr;
  const uint32_t n = t->n_tables, m = n_maps;
  const std::string_view tx(text ? text : "", text_len);
  // py:1690-1699: the text, then every key, then every value, all states in one batch
  Strs in;
  for (uint32_t s = 0; s < n; s++) {
    in.add(tx, s);
    for (uint32_t j = 0; j < m; j++) in.add(std::string_view(maps[j].key, maps[j].key_len), s);
    for (uint32_t j = 0; j < m; j++) in.add(std::string_view(maps[j].value, maps[j].value_len), s);
  }
  Trace tr("goto");
  tr.mark("pack", in.size());
  Res r;
  int rc = interp(x, t, in, r);
  if (rc) return rc;
  tr.mark("interp", in.size());
  MapOut o;
  o.status.reserve(n);
  Blocks blocks;
  Strs texts;
  std::vector<uint32_t> range, pend, fail_at;
  std::vector<std::string> keys(m);
  std::vector<uint8_t> st(n, IE_OK_STR);
  std::vector<uint32_t> wh(n, 0);
  std::vector<int32_t> ch(n, -1);
  const bool rs = t->dialect == IE_DIALECT_RS;
  for (uint32_t s = 0; s < n; s++) {
    const uint64_t b = (uint64_t)s * (1 + 2 * m);
    const uint8_t ts = r.st[b];
    if (rs) {
      // runtime.rs:1093-1129: any error of the text takes the NULL branch; the maps are tried in
      // order, a key (and, when the text resolved, its value) interpolated only when reached
      if (!ok(ts)) {
        for (uint32_t j = 0; j < m && ch[s] < 0 && st[s] == IE_OK_STR; j++) {
          if (!ok(r.st[b + 1 + j])) st[s] = r.st[b + 1 + j], wh[s] = 1 + j;
          else if (r.text[b + 1 + j] == "NULL") {
            if (!ok(r.st[b + 1 + m + j])) st[s] = r.st[b + 1 + m + j], wh[s] = 1 + m + j;
            else ch[s] = (int32_t)j;
          }
        }
        if (ch[s] < 0 && st[s] == IE_OK_STR) st[s] = IE_E_NO_NULL;
        continue;
      }
      uint32_t f = m;  // the first map whose key or value fails: the maps before it can match
      for (uint32_t j = 0; j < m && f == m; j++)
        if (!ok(r.st[b + 1 + j]) || !ok(r.st[b + 1 + m + j])) f = j;
      for (uint32_t j = 0; j < f; j++) keys[j].assign(r.text[b + 1 + j]);
      const auto rg = blocks.range(keys, f);
      range.push_back(rg.first);
      range.push_back(rg.second);
      texts.add(r.text[b], s);
      pend.push_back(s);
      fail_at.push_back(f);
      continue;
    }
    if (!ok(ts) && ts != IE_E_INTERP) {  // py:1693 catches InterpolationException only
      st[s] = ts;
      continue;
    }
    uint32_t bad = 0;
    for (uint32_t j = 0; j < 2 * m && !bad; j++)  // py:1698-1699: the first failing key, then value
      if (!ok(r.st[b + 1 + j])) bad = 1 + j;
    if (bad) {
      st[s] = r.st[b + bad];
      wh[s] = bad;
      continue;
    }
    if (ts == IE_E_INTERP) {  // py:1702-1705: the 'NULL' key's value
      for (uint32_t j = 0; j < m && ch[s] < 0; j++)
        if (r.text[b + 1 + j] == "NULL") ch[s] = (int32_t)j;
      if (ch[s] < 0) st[s] = IE_E_NO_NULL;
      continue;
    }
    for (uint32_t j = 0; j < m; j++) keys[j].assign(r.text[b + 1 + j]);
    const auto rg = blocks.range(keys, m);
    range.push_back(rg.first);
    range.push_back(rg.second);
    texts.add(r.text[b], s);
    pend.push_back(s);
    fail_at.push_back(m);
  }
  tr.mark("blocks", blocks.pats.size());
  Match mt;
  if ((rc = match_first(x, t, blocks.pats, texts, range, mt))) return rc;
  tr.mark("match", texts.size());
  for (size_t k = 0; k < pend.size(); k++) {  // py:1707-1709: the first key matching the text
    const uint32_t s = pend[k];
    const uint64_t b = (uint64_t)s * (1 + 2 * m);
    if (mt.match[k] >= 0) {
      ch[s] = mt.match[k] - (int32_t)range[2 * k];
    } else if (fail_at[k] < m) {  // (rs: no match before the first failing map: its error)
      const uint32_t f = fail_at[k];
      const bool key_bad = !ok(r.st[b + 1 + f]);
      st[s] = key_bad ? r.st[b + 1 + f] : r.st[b + 1 + m + f];
      wh[s] = key_bad ? 1 + f : 1 + m + f;
    } else {
      st[s] = IE_E_NO_MATCH;
    }
  }
  for (uint32_t s = 0; s < n; s++) {
    const uint64_t b = (uint64_t)s * (1 + 2 * m);
    if (st[s] == IE_OK_STR) o.push(r.text[b + 1 + m + ch[s]], IE_OK_STR, 0, ch[s]);
    else o.push(st[s] == IE_E_NO_MATCH ? std::string_view(r.text[b]) : std::string_view(), st[s], wh[s], -1);  // (py:1708 names the text)
  }
  rc = emit(o, out);
  tr.mark("emit", n);
  return rc;
}

int ie_replace_map(ie_exec* x, const ie_table* t, const char* name, uint64_t name_len, const uint8_t* bytes,
                   const uint64_t* offsets, const uint32_t* table_id, uint64_t n, const ie_map_pair* maps,
                   uint32_t n_maps, int32_t repeat_until_done, ie_map_result** names, ie_map_result** out) {
  if (!x || !t || !out || (n && (!bytes || !offsets || !table_id)) || (n_maps && !maps) || (name && !names))
    return fail(IE_ERR_INVALID, "null argument");
  *out = nullptr;
  if (names) *names = nullptr;
  for (uint64_t i = 0; i < n; i++)
    if (table_id[i] >= t->n_tables) return fail(IE_ERR_INVALID, "table id beyond the table set");
  const uint32_t m = n_maps, nt = t->n_tables;
  std::vector<std::string_view> rk(m), rv(m);
  bool live_keys = false;  // a key text holds a brace: interpolated again on every pass (py:1728)
  for (uint32_t j = 0; j < m; j++) {
    rk[j] = std::string_view(maps[j].key, maps[j].key_len);
    rv[j] = std::string_view(maps[j].value, maps[j].value_len);
    live_keys |= rk[j].find('{') != std::string_view::npos;
  }
  // each leaf's text between passes (a pass reads it into its batch, and writes it once at its end)
  std::vector<std::string> cur(n);
  for (uint64_t i = 0; i < n; i++) cur[i] = std::string((const char*)bytes + offsets[i], offsets[i + 1] - offsets[i]);
  // the owners' interpolated keys (per state: the keys before the first that fails, and its status)
  std::vector<std::vector<std::string>> keys(nt);
  std::vector<uint32_t> key_ok(nt, m), key_at(nt, UINT32_MAX);
  std::vector<uint8_t> key_st(nt, IE_OK_STR);
  std::vector<uint8_t> st(n, IE_OK_STR);
  std::vector<uint32_t> wh(n, 0);
  std::vector<int32_t> ch(n, -1);
  std::vector<uint64_t> active(n);
  for (uint64_t i = 0; i < n; i++) active[i] = i;
  MapOut nm;
  Trace tr("replace");
  int rc = IE_SUCCESS;
  if (name && n == 0) {  // output_name alone (no leaves to run)
    Strs in;
    for (uint32_t s = 0; s < nt; s++) in.add(std::string_view(name, name_len), s);
    Res r;
    if ((rc = interp(x, t, in, r))) return rc;
    for (uint32_t s = 0; s < nt; s++)
      nm.push(ok(r.st[s]) ? std::string_view(r.text[s]) : std::string_view(), r.st[s], 0, -1, r.vid[s]);
  }
  for (uint32_t pass = 1; !active.empty(); pass++) {
    if (pass > kMaxPasses) {  // the reference spins forever
      for (uint64_t i : active) st[i] = IE_DIVERGED;
      break;
    }
    // 1. interpolate (py:1722); the keys of this pass (py:1728); on the first pass output_name (py:1715)
    Strs in;
    {
      uint64_t nb = 0;
      for (uint64_t i : active) nb += cur[i].size();
      in.reserve(active.size() + (uint64_t)nt * m + (name ? nt : 0), nb + 64 * (uint64_t)nt * m);
    }
    for (uint64_t i : active) in.add(cur[i], table_id[i]);
    std::vector<uint32_t> kst;
    if (pass == 1 || live_keys) {
      std::vector<bool> seen(nt, false);
      for (uint64_t i : active)
        if (!seen[table_id[i]]) seen[table_id[i]] = true, kst.push_back(table_id[i]);
      std::sort(kst.begin(), kst.end());
      for (uint32_t s : kst)
        for (uint32_t j = 0; j < m; j++) in.add(rk[j], s);
    }
    const uint64_t name0 = in.size();
    if (pass == 1 && name)
      for (uint32_t s = 0; s < nt; s++) in.add(std::string_view(name, name_len), s);
    tr.mark("pack", in.size());
    Res r;
    if ((rc = interp(x, t, in, r))) return rc;
    tr.mark("interp", in.size());
    if (pass == 1 && name) {  // no str(): a typed output_name stays typed (py:1715)
      for (uint32_t s = 0; s < nt; s++) {
        const uint64_t k = name0 + s;
        nm.push(ok(r.st[k]) ? std::string_view(r.text[k]) : std::string_view(), r.st[k], 0, -1, r.vid[k]);
      }
    }
    for (size_t q = 0; q < kst.size(); q++) {
      const uint32_t s = kst[q];
      keys[s].assign(m, std::string());
      key_ok[s] = m;
      for (uint32_t j = 0; j < m; j++) {
        const uint64_t k = active.size() + (uint64_t)q * m + j;
        if (!ok(r.st[k])) {
          key_ok[s] = j;
          key_st[s] = r.st[k];
          break;
        }
        keys[s][j].assign(r.text[k]);
      }
    }
    // the strings that interpolated: their batch position (the pass's starting text, for the fixed
    // point) and their text, as views (of this pass's batch and results, alive until its end)
    std::vector<uint64_t> alive, alive_q;
    std::vector<std::string_view> iv;
    uint64_t alive_bytes = 0;
    alive.reserve(active.size());
    alive_q.reserve(active.size());
    iv.reserve(active.size());
    for (size_t q = 0; q < active.size(); q++) {
      const uint64_t i = active[q];
      if (!ok(r.st[q])) {
        st[i] = r.st[q];  // (cur[i]: the string that failed)
        continue;
      }
      alive.push_back(i);
      alive_q.push_back(q);
      iv.push_back(r.text[q]);
      alive_bytes += r.text[q].size();
    }
    // 2. the first map whose key matches (py:1725-1735), every leaf in one launch
    Blocks blocks;
    Strs mstr;
    mstr.reserve(alive.size(), alive_bytes);
    std::vector<uint32_t> range;
    range.reserve(2 * alive.size());
    std::unordered_map<uint32_t, std::pair<uint32_t, uint32_t>> rg_of;  // (a state's leaves share its block)
    for (size_t k = 0; k < alive.size(); k++) {
      const uint32_t s = table_id[alive[k]];
      auto it = rg_of.find(s);
      if (it == rg_of.end()) it = rg_of.emplace(s, blocks.range(keys[s], key_ok[s])).first;
      const auto rg = it->second;
      range.push_back(rg.first);
      range.push_back(rg.second);
      mstr.add(iv[k], s);
    }
    tr.mark("blocks", blocks.pats.size());
    Match mt;
    if ((rc = match_first(x, t, blocks.pats, mstr, range, mt))) return rc;
    tr.mark("match", mstr.size());
    // 3. the matched maps' values against inserts | {'1': capture, ...} (py:1732-1738)
    Strs vin;                                // captures spliced in, on the states' own tables
    std::vector<uint64_t> vleaf;             // (positions in `alive`)
    std::vector<uint32_t> slow_owner;        // the rest: a table of their own
    std::vector<std::vector<std::pair<std::string, std::string>>> slow_extra;
    std::vector<uint64_t> slow_leaf;
    Strs sin;
    for (size_t q = 0; q < alive.size(); q++) {
      const uint64_t i = alive[q];
      const uint32_t s = table_id[i];
      if (mt.match[q] < 0) {
        if (key_ok[s] < m) {  // a key failed before anything matched: its error propagates
          st[i] = key_st[s];
          wh[i] = 1 + key_ok[s];
        }
        continue;
      }
      const uint32_t j = (uint32_t)mt.match[q] - range[2 * q];
      ch[i] = (int32_t)j;
      std::vector<std::string_view> caps(mt.ncap[q]);
      bool inert = true;
      for (uint32_t c = 0; c < mt.ncap[q]; c++) {
        const uint32_t a = mt.caps[(q * IE_WC_MAX_CAP + c) * 2], l = mt.caps[(q * IE_WC_MAX_CAP + c) * 2 + 1];
        caps[c] = iv[q].substr(a, l);
        inert &= (text_flags(caps[c]) & EF_INERT) != 0;
      }
      if (inert && substitutable(rv[j])) {
        if (caps.empty()) {
          vin.add(rv[j], s);
        } else {  // (the substituted value straight into the batch)
          substitute(vin.bytes, rv[j], caps);
          vin.off.push_back(vin.bytes.size());
          vin.tid.push_back(s);
        }
        vleaf.push_back(q);
      } else {
        std::vector<std::pair<std::string, std::string>> ex;
        for (uint32_t c = 0; c < caps.size(); c++) ex.emplace_back(std::to_string(c + 1), std::string(caps[c]));
        sin.add(rv[j], (uint32_t)slow_owner.size());
        slow_owner.push_back(s);
        slow_extra.push_back(std::move(ex));
        slow_leaf.push_back(q);
      }
    }
    tr.mark("captures", vin.size());
    Res vr;
    if ((rc = interp(x, t, vin, vr))) return rc;
    tr.mark("values", vin.size());
    // each alive string's text at the end of the pass: its value's, or (no match, a failed value:
    // the matched text) the interpolated one
    std::vector<std::string_view> nv(iv);
    for (size_t q = 0; q < vleaf.size(); q++) {
      const uint64_t i = alive[vleaf[q]];
      if (!ok(vr.st[q])) st[i] = vr.st[q], wh[i] = 1 + m + (uint32_t)ch[i];
      else nv[vleaf[q]] = vr.text[q];
    }
    Res sr;
    if (!slow_owner.empty()) {
      ie_table* xt = nullptr;
      if ((rc = table_with(x, t, slow_owner, slow_extra, &xt))) return rc;
      rc = interp(x, xt, sin, sr);
      ie_table_free(xt);
      if (rc) return rc;
      for (size_t q = 0; q < slow_leaf.size(); q++) {
        const uint64_t i = alive[slow_leaf[q]];
        if (!ok(sr.st[q])) st[i] = sr.st[q], wh[i] = 1 + m + (uint32_t)ch[i];
        else nv[slow_leaf[q]] = sr.text[q];
      }
      tr.mark("slow values", sin.size());
    }
    // 4. the pass's texts kept; a fixed point (against the text the pass started from, still in its
    // batch), or one pass without repeat_until_done (py:1742-1745)
    std::vector<uint64_t> next;
    for (size_t k = 0; k < alive.size(); k++) {
      const uint64_t i = alive[k], q = alive_q[k];
      cur[i].assign(nv[k]);
      if (st[i] != IE_OK_STR || !repeat_until_done) continue;
      const std::string_view start((const char*)in.bytes.data() + in.off[q], in.off[q + 1] - in.off[q]);
      if (start != std::string_view(cur[i])) next.push_back(i);
    }
    active.swap(next);
  }
  MapOut o;
  {
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) total += cur[i].size();
    o.bytes.reserve(total);
  }
  for (uint64_t i = 0; i < n; i++) o.push(cur[i], st[i], st[i] == IE_OK_STR ? 0u : wh[i], ch[i]);
  if (name) emit(nm, names);
  rc = emit(o, out);
  tr.mark("emit", n);
  return rc;
}

int ie_delete_keys(ie_exec* x, ie_table* t, const uint32_t* states, uint32_t n_states, const uint8_t* wbytes,
                   const uint64_t* woffsets, uint32_t n_wildcards, int32_t except_matching, ie_map_result** out) {
  if (!x || !t || !out || (n_states && !states) ||
      (n_wildcards && (!woffsets || (!wbytes && woffsets[n_wildcards] > woffsets[0]))))
    return fail(IE_ERR_INVALID, "null argument");
  *out = nullptr;
  std::vector<bool> in(t->n_tables, states == nullptr);
  for (uint32_t k = 0; k < n_states; k++) {
    if (states[k] >= t->n_tables) return fail(IE_ERR_INVALID, "state beyond the table set");
    in[states[k]] = true;
  }
  // every key of the states (not the clock entries: the table's, never a dict key), in slot order
  Strs ks;
  for (uint32_t s = 0; s < (uint32_t)t->h_entries.size(); s++) {
    const Entry& e = t->h_entries[s];
    if (!(e.flags & EF_OCCUPIED) || e.vid >= IE_VID_CLOCK_HHMMSS || !in[e.flags >> kTidShift]) continue;
    ks.add(mirror_key(t, e), e.flags >> kTidShift);
  }
  std::vector<std::string> pats;
  for (uint32_t w = 0; w < n_wildcards; w++)
    pats.emplace_back((const char*)wbytes + woffsets[w], woffsets[w + 1] - woffsets[w]);
  Match mt;
  int rc = match_first(x, t, pats, ks, {}, mt);
  if (rc) return rc;
  // delete: the keys some wildcard matches (py:1843-1855); delete_except: the others (py:1857-1868)
  MapOut o;
  std::vector<ie_kv> kv;
  std::vector<uint32_t> tids, vids;
  for (uint64_t k = 0; k < ks.size(); k++) {
    if ((mt.match[k] >= 0) == (except_matching != 0)) continue;
    const std::string_view key((const char*)ks.bytes.data() + ks.off[k], ks.off[k + 1] - ks.off[k]);
    o.push(key, IE_OK_STR, ks.tid[k], -1);
  }
  // (keys copied out first: the update rewrites the mirror they point into). The store path
  // (ie_table_set_store) gives each deleted key's value id back to the table's free list and
  // reports it, so the caller drops the value it held under that id (value_id in the result)
  for (uint64_t k = 0; k < o.status.size(); k++) {
    kv.push_back(ie_kv{(const char*)o.bytes.data() + o.off[k], o.off[k + 1] - o.off[k], nullptr, 0, -1, 0});
    tids.push_back(o.where[k]);
    vids.push_back(IE_VID_NONE);
  }
  if (!kv.empty() && (rc = ie_table_set_store(t, kv.data(), tids.data(), kv.size(), vids.data()))) return rc;
  for (uint64_t k = 0; k < vids.size(); k++) o.vid[k] = vids[k];
  return emit(o, out);
}

}  // extern "C"
