// cld_dynamic_data.cpp -- CLD2 dynamic data file ("cld2_data_file00") -> CLDT.
//
// The reference can load its scoring tables at run time from a data file
// instead of linking them (CLD2_DYNAMIC_MODE):
//   format      cld2/internal/cld2_dynamic_data.h:22-147
//   header size cld2/internal/cld2_dynamic_data.cc:45-49
//   loader      cld2/internal/cld2_dynamic_data_loader.cc:41-146 (header),
//               :196-270 (tables)
//   writer      cld2/internal/cld2_dynamic_data_extractor.cc:45-195, 199-290
// The file carries exactly the ScoringTables fields (scoreonescriptspan.h:100-114):
// the CJK unigram property machine (unigram_obj), kAvgDeltaOctaScore and seven
// CLD2TableSummary tables in the fixed order compat, deltabi, distinctbi,
// quadgram, quadgram2, deltaocta, distinctocta (loader :253-260).  Everything
// else the hot path reads (script/lowercase/scan machines, kLgProbV2Tbl, the
// language/script maps) is compiled into CLD2 in both modes, so it is taken
// from a base CLDT blob.  This is how a user-supplied real quadchrome table
// reaches the GPU: no rebuild, no code generation.
//
// Validation is the loader's (marker, exact header size, total size equal to
// the file size) plus what the loader leaves unchecked and a GPU gather would
// turn into an out-of-bounds read: every block inside the file, bucket counts
// matching kCLDTableSize, power-of-two table sizes, and every indirect index a
// bucket can produce inside kCLDTableInd (the same bound the table extractor
// asserts, oracle/tablegen/extract_cld2_tables.cc emit_summary).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <utility>
#include <vector>

#include "cld_dynamic_data.h"
#include "cldt_format.h"

namespace cld {
namespace {

constexpr char kMarker[16] = {'c', 'l', 'd', '2', '_', 'd', 'a', 't', 'a', '_', 'f', 'i', 'l', 'e', '0', '0'};
constexpr uint32_t kNumTables = 7;
constexpr uint32_t kTableIds[kNumTables] = {CLDT_CJK_COMPAT, CLDT_DELTA_BI, CLDT_DISTINCT_BI, CLDT_QUAD,
                                            CLDT_QUAD2, CLDT_DELTA_OCTA, CLDT_DISTINCT_OCTA};

uint32_t header_size(uint32_t n_tables) { return 16 + 20 * 4 + n_tables * 10 * 4; }   // cld2_dynamic_data.cc:45-49

struct Reader {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  uint32_t u32() {
    if (pos + 4 > n) { ok = false; return 0; }
    uint32_t v;
    memcpy(&v, p + pos, 4);
    pos += 4;
    return v;
  }
};

void put(std::vector<uint8_t>& o, const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  o.insert(o.end(), b, b + n);
}
void pad16(std::vector<uint8_t>& o) { while (o.size() % 16) o.push_back(0); }

bool in_file(uint64_t start, uint64_t len, size_t file) { return start <= file && len <= file - start; }

}  // namespace

int cld2_data_to_cldt(const uint8_t* data, size_t len, const uint8_t* base, size_t base_len,
                      std::vector<uint8_t>* out, std::string* err) {
  auto fail = [&](const std::string& m) { if (err) *err = m; return -22; };
  if (!data || len < 16 || memcmp(data, kMarker, 16) != 0) return fail("Malformed header: bad file marker");
  Reader r{data, len, 16};
  const uint32_t total = r.u32();
  struct { uint32_t state0, state0_size, total_size, max_expand, entry_shift, bytes_per_entry, losub, hiadd; } u;
  u.state0 = r.u32(); u.state0_size = r.u32(); u.total_size = r.u32(); u.max_expand = r.u32();
  u.entry_shift = r.u32(); u.bytes_per_entry = r.u32(); u.losub = r.u32(); u.hiadd = r.u32();
  uint32_t st_off = r.u32(), st_len = r.u32();
  r.u32(); r.u32();                       // remap_base: unused by property lookups (GetUniHits)
  r.u32(); r.u32();                       // remap_string: likewise
  r.u32(); r.u32();                       // fast_state: likewise
  const uint32_t es_off = r.u32(), es_len = r.u32();
  const uint32_t n_tables = r.u32();
  if (!r.ok) return fail("truncated header");
  if (n_tables != kNumTables)             // loader :253-260 dereferences exactly 7 tables
    return fail("expected 7 tables, file has " + std::to_string(n_tables));
  struct TH { uint32_t size_one, size, key_mask, build_date, t_off, t_len, i_off, i_len, s_off, s_len; } th[kNumTables];
  for (auto& t : th) {
    t.size_one = r.u32(); t.size = r.u32(); t.key_mask = r.u32(); t.build_date = r.u32();
    t.t_off = r.u32(); t.t_len = r.u32(); t.i_off = r.u32(); t.i_len = r.u32(); t.s_off = r.u32(); t.s_len = r.u32();
  }
  if (!r.ok || r.pos != header_size(n_tables))
    return fail("Header size mismatch");
  if (total != len) return fail("File size mismatch");
  // unigram_obj: a one-byte-entry property machine (UTF8GenericPropertyBigOneByte, utf8statetable.cc:271-320)
  if (u.bytes_per_entry != 1 || st_len != u.total_size || !in_file(st_off, st_len, len) || st_off < r.pos)
    return fail("bad unigram state table block");
  if (u.state0 >= u.total_size || u.state0_size > u.total_size || u.entry_shift > 16 ||
      ((uint64_t)(u.total_size - 1) >> u.entry_shift) > 0xFFFFFF)
    return fail("bad unigram state machine parameters");
  if (es_len % 2 || !in_file(es_off, es_len, len) || es_off < r.pos) return fail("bad kAvgDeltaOctaScore block");

  // ---- base blob sections
  if (!base || base_len < sizeof(cldt_file_header)) return fail("bad base CLDT blob");
  cldt_file_header fh;
  memcpy(&fh, base, sizeof(fh));
  if (fh.magic != CLDT_MAGIC || fh.version != CLDT_VERSION ||
      !in_file(fh.section_table_offset, (uint64_t)fh.n_sections * sizeof(cldt_section), base_len))
    return fail("bad base CLDT blob");
  std::vector<std::pair<uint32_t, std::vector<uint8_t>>> secs;
  for (uint32_t i = 0; i < fh.n_sections; ++i) {
    cldt_section s;
    memcpy(&s, base + fh.section_table_offset + i * sizeof(cldt_section), sizeof(s));
    if (!in_file(s.offset, s.size, base_len)) return fail("bad base CLDT section");
    secs.emplace_back(s.id, std::vector<uint8_t>(base + s.offset, base + s.offset + s.size));
  }
  auto replace = [&](uint32_t id, std::vector<uint8_t>&& b) {
    for (auto& s : secs) if (s.first == id) { s.second = std::move(b); return true; }
    return false;
  };

  {  // CJK unigram machine
    std::vector<uint8_t> b;
    cldt_sm_header h;
    memset(&h, 0, sizeof(h));
    h.state0 = u.state0; h.state0_size = u.state0_size; h.total_size = u.total_size;
    h.entry_shift = u.entry_shift; h.bytes_per_entry = 1; h.losub = u.losub; h.hiadd = u.hiadd;
    put(b, &h, sizeof(h));
    put(b, data + st_off, st_len);
    pad16(b);
    if (!replace(CLDT_CJK_UNI_PROP, std::move(b))) return fail("base blob lacks the unigram machine");
  }
  {  // kAvgDeltaOctaScore: the base's size fixes the language count the kernels index with
    std::vector<uint8_t> b(data + es_off, data + es_off + es_len);
    if (!replace(CLDT_EXPECTED_SCORE, std::move(b))) return fail("base blob lacks kAvgDeltaOctaScore");
  }
  for (uint32_t k = 0; k < kNumTables; ++k) {
    const TH& t = th[k];
    if ((uint64_t)t.size * 16 != t.t_len || !in_file(t.t_off, t.t_len, len) || !in_file(t.i_off, t.i_len, len) ||
        t.i_len % 4 || (t.size & (t.size - 1)) != 0 || (t.size && t.t_off < r.pos))
      return fail("table " + std::to_string(k) + ": bad block");
    const uint32_t n_ind = t.i_len / 4;
    const uint32_t n_b = t.size ? t.size : 1;   // a size-0 table still owns one (empty) bucket
    std::vector<uint8_t> buckets((size_t)n_b * 16, 0);
    if (t.size) memcpy(buckets.data(), data + t.t_off, t.t_len);
    for (uint32_t i = 0; i < n_b * 4; ++i) {       // every reachable indirect must be inside kCLDTableInd
      uint32_t kv;
      memcpy(&kv, buckets.data() + 4 * i, 4);
      if (kv == 0) continue;
      const uint32_t ind = kv & ~t.key_mask;
      const uint64_t need = ind < t.size_one ? (uint64_t)ind + 1 : (uint64_t)ind + (ind - t.size_one) + 2;
      if (need > n_ind) return fail("table " + std::to_string(k) + ": indirect index beyond kCLDTableInd");
    }
    std::vector<uint8_t> b;
    cldt_table_header h;
    memset(&h, 0, sizeof(h));
    h.size_one = t.size_one; h.size = t.size; h.key_mask = t.key_mask; h.build_date = t.build_date;
    h.n_ind = n_ind; h.n_buckets_stored = n_b;
    put(b, &h, sizeof(h));
    put(b, buckets.data(), buckets.size());
    put(b, data + t.i_off, t.i_len);
    if (!replace(kTableIds[k], std::move(b))) return fail("base blob lacks table " + std::to_string(k));
  }
  {  // provenance note
    std::string note = "tables: cld2 dynamic data file (" + std::to_string(len) + " bytes) over the base CLDT";
    std::vector<uint8_t> b(note.begin(), note.end());
    if (!replace(CLDT_PROVENANCE, std::move(b))) secs.emplace_back(CLDT_PROVENANCE, std::move(b));
  }

  // ---- serialise (same layout rules as tools/cldt.py write_blob)
  std::vector<uint8_t>& o = *out;
  o.assign(32, 0);
  std::vector<cldt_section> table;
  for (auto& s : secs) {
    pad16(o);
    cldt_section e;
    memset(&e, 0, sizeof(e));
    e.id = s.first; e.offset = o.size(); e.size = s.second.size();
    table.push_back(e);
    put(o, s.second.data(), s.second.size());
  }
  pad16(o);
  cldt_file_header nh;
  memset(&nh, 0, sizeof(nh));
  nh.magic = CLDT_MAGIC; nh.version = CLDT_VERSION; nh.n_sections = (uint32_t)table.size();
  nh.section_table_offset = o.size();
  put(o, table.data(), table.size() * sizeof(cldt_section));
  memcpy(o.data(), &nh, sizeof(nh));
  return 0;
}

}  // namespace cld
