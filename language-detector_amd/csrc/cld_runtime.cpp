// cld_runtime.cpp -- host runtime behind the C ABI (include/cld_mi355x.h).
//
//  * loads the CLDT table blob once per process, uploads it once per GPU;
//  * one context per GPU: stream, table copy, general-kernel arena, staging;
//  * cld_detect_batch shards documents across GPUs by byte count (documents
//    are independent: no collective on the hot path), one host thread per GPU;
//  * detect_language() (wrapper.h:8) coalesces concurrent callers into GPU
//    micro-batches.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "cld_coalesce.h"
#include "cld_dlqueue.h"
#include "cld_device.h"
#include "cld_dynamic_data.h"
#include "cld_hints.h"
#include "cld_kernels.h"
#include "cldt_format.h"

namespace {

// Inside a loop that has enqueued DMA on the caller's buffers: record the
// error and leave the loop, so the drain after it still runs.
#define HIP_BRK(x)                                                          \
  if (hipError_t e_ = (x); e_ != hipSuccess) {                              \
    fprintf(stderr, "cld_mi355x: %s failed: %s (%s:%d)\n", #x,              \
            hipGetErrorString(e_), __FILE__, __LINE__);                     \
    rc = CLD_EFAULT;                                                        \
    break;                                                                  \
  }

#define HIP_OK(x)                                                           \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "cld_mi355x: %s failed: %s (%s:%d)\n", #x,            \
              hipGetErrorString(e_), __FILE__, __LINE__);                   \
      return CLD_EFAULT;                                                    \
    }                                                                       \
  } while (0)

// offsets[0..n] non-decreasing: a branch-free pass the compiler vectorises
// (an early exit per element kept it scalar: ~0.5 ms per million documents
// of every batch call)
bool offsets_nondecreasing(const uint64_t* offsets, size_t n) {
  uint64_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad |= (uint64_t)(offsets[i + 1] < offsets[i]);
  return bad == 0;
}

// ------------------------------------------------------------ host tables
// Language codes and names handed to callers stay valid for the life of the
// process (the reference returns static strings, lang_script.cc:205-217):
// they are interned once and never freed, even when the tables are swapped.
const char* intern(const std::string& v) {
  static std::mutex mu;
  static std::set<std::string>* pool = new std::set<std::string>();
  std::lock_guard<std::mutex> lk(mu);
  return pool->insert(v).first->c_str();
}

struct HostTables {
  std::vector<uint8_t> blob;
  cldt_meta meta{};
  std::vector<const char*> codes, names;   // interned
  std::string version;
  DevTables offs{};   // pointer fields hold byte offsets into blob
  cld::HintView hints;   // host views for cld_hint_priors (null fields: the blob has no hint sections)
};

// Section `id` of a parsed blob; parse_tables has checked that every section
// table entry lies inside the blob before any other reader runs.
const uint8_t* section(const std::vector<uint8_t>& b, uint32_t id, uint64_t* off, uint64_t* size) {
  const cldt_file_header* fh = (const cldt_file_header*)b.data();
  const cldt_section* s = (const cldt_section*)(b.data() + fh->section_table_offset);
  for (uint32_t i = 0; i < fh->n_sections; ++i)
    if (s[i].id == id) {
      if (off) *off = s[i].offset;
      if (size) *size = s[i].size;
      return b.data() + s[i].offset;
    }
  return nullptr;
}

template <class P>
P at(uint64_t off) { return reinterpret_cast<P>((uintptr_t)off); }

bool parse_sm(const std::vector<uint8_t>& b, uint32_t id, DevSM* sm) {
  uint64_t off, size;
  const uint8_t* p = section(b, id, &off, &size);
  if (!p || size < sizeof(cldt_sm_header)) return false;
  const cldt_sm_header* h = (const cldt_sm_header*)p;
  if (h->bytes_per_entry != 1 && h->bytes_per_entry != 2) return false;
  sm->state0 = h->state0; sm->state0_size = h->state0_size; sm->total = h->total_size;
  sm->shift = h->entry_shift; sm->n_remap = h->n_remap; sm->n_rstr = h->n_remap_string;
  uint64_t tbl = off + sizeof(cldt_sm_header);
  if (h->bytes_per_entry == 2) {
    sm->t16 = at<const uint16_t*>(tbl); sm->t8 = nullptr;
  } else {
    sm->t8 = at<const uint8_t*>(tbl); sm->t16 = nullptr;
  }
  uint64_t r = (sizeof(cldt_sm_header) + (uint64_t)h->total_size * h->bytes_per_entry + 15) & ~15ull;
  sm->remap = at<const uint8_t*>(off + r);
  sm->rstr = at<const uint8_t*>(off + r + 4ull * h->n_remap);
  // every table entry, remap entry and remap byte the machines can index lies inside the section
  // (the device bounds each table read by `total`)
  const uint64_t need = h->bytes_per_entry == 2 ? sizeof(cldt_sm_header) + 2ull * h->total_size
                                                : r + 4ull * h->n_remap + h->n_remap_string;
  return need <= size && h->state0 < h->total_size;
}

bool parse_tbl(const std::vector<uint8_t>& b, uint32_t id, DevTbl* t) {
  uint64_t off, size;
  const uint8_t* p = section(b, id, &off, &size);
  if (!p || size < sizeof(cldt_table_header)) return false;
  const cldt_table_header* h = (const cldt_table_header*)p;
  t->size_one = h->size_one; t->size = h->size; t->key_mask = h->key_mask;
  t->n_ind = h->n_ind; t->n_buckets = h->n_buckets_stored;
  uint64_t bo = off + sizeof(cldt_table_header);
  t->b = at<const uint32_t*>(bo);
  t->ind = at<const uint32_t*>(bo + 16ull * h->n_buckets_stored);
  // buckets are read as one 16-byte vector: they must be 16-byte aligned; the
  // subscript is masked with size-1, so every such bucket must be stored; the
  // indirect reads are bounded by n_ind on the device
  return (bo % 16) == 0 && (h->size == 0 || (h->size & (h->size - 1)) == 0) &&
         h->size <= h->n_buckets_stored &&
         sizeof(cldt_table_header) + 16ull * h->n_buckets_stored + 4ull * h->n_ind <= size;
}

std::vector<std::string> strings(const std::vector<uint8_t>& b, uint32_t id) {
  std::vector<std::string> out;
  uint64_t size = 0;
  const uint8_t* p = section(b, id, nullptr, &size);
  if (!p || size < 4) return out;
  uint32_t n = *(const uint32_t*)p;
  if (4ull * (n + 2) > size) return out;
  const uint32_t* o = (const uint32_t*)(p + 4);
  const char* base = (const char*)(p + 4 + 4 * (n + 1));
  const uint64_t avail = size - 4ull * (n + 2);
  for (uint32_t i = 0; i < n; ++i) {
    if (o[i] >= avail) return std::vector<std::string>();
    out.emplace_back(base + o[i], strnlen(base + o[i], avail - o[i]));
  }
  return out;
}

int read_file(const char* path, std::vector<uint8_t>* out) {
  FILE* f = fopen(path, "rb");
  if (!f) return CLD_EINVAL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (n < 0) { fclose(f); return CLD_EIO; }
  out->resize((size_t)n);
  size_t got = fread(out->data(), 1, (size_t)n, f);
  fclose(f);
  return got == (size_t)n ? CLD_OK : CLD_EIO;
}

// Parse a CLDT blob (already in t->blob) into table offsets; `label` names it in cld_version().
int parse_tables(HostTables* t, const std::string& label) {
  const long n = (long)t->blob.size();
  if (n < (long)sizeof(cldt_file_header)) return CLD_EINVAL;
  const cldt_file_header* fh = (const cldt_file_header*)t->blob.data();
  if (fh->magic != CLDT_MAGIC || fh->version != CLDT_VERSION || fh->n_sections > 4096 ||
      fh->section_table_offset + (uint64_t)fh->n_sections * sizeof(cldt_section) > (uint64_t)n)
    return CLD_EINVAL;
  {  // every section lies inside the blob and is 4-byte aligned (the tables are read as u16/u32/u64)
    const cldt_section* sec = (const cldt_section*)(t->blob.data() + fh->section_table_offset);
    for (uint32_t i = 0; i < fh->n_sections; ++i)
      if (sec[i].offset > (uint64_t)n || sec[i].size > (uint64_t)n - sec[i].offset || sec[i].offset % 4)
        return CLD_EINVAL;
  }
  uint64_t msize = 0;
  const uint8_t* m = section(t->blob, CLDT_META, nullptr, &msize);
  if (!m || msize < sizeof(t->meta)) return CLD_EINVAL;
  memcpy(&t->meta, m, sizeof(t->meta));
  DevTables& D = t->offs;
  bool ok = parse_sm(t->blob, CLDT_SCRIPT_PROP, &D.script) && parse_sm(t->blob, CLDT_LOWER_REPL, &D.lower) &&
            parse_sm(t->blob, CLDT_SCAN_NOT, &D.scan) && parse_sm(t->blob, CLDT_CJK_UNI_PROP, &D.uni) &&
            parse_tbl(t->blob, CLDT_CJK_COMPAT, &D.compat) && parse_tbl(t->blob, CLDT_DELTA_BI, &D.deltabi) &&
            parse_tbl(t->blob, CLDT_DISTINCT_BI, &D.distinctbi) && parse_tbl(t->blob, CLDT_QUAD, &D.quad) &&
            parse_tbl(t->blob, CLDT_QUAD2, &D.quad2) && parse_tbl(t->blob, CLDT_DELTA_OCTA, &D.deltaocta) &&
            parse_tbl(t->blob, CLDT_DISTINCT_OCTA, &D.distinctocta);
  if (!ok) return CLD_EINVAL;
  uint64_t off, size;
  struct { uint32_t id; const void** dst; uint32_t* count; uint32_t elem; } secs[] = {
      {CLDT_EXPECTED_SCORE, (const void**)&D.expected, &D.n_expected, 2},
      {CLDT_LGPROB, (const void**)&D.lgprob, nullptr, 1},
      {CLDT_LANG_TO_PLANG, (const void**)&D.l2p, &D.l2p_size, 1},
      {CLDT_PLANG_TO_LANG_LATN, (const void**)&D.p2l_latn, nullptr, 2},
      {CLDT_PLANG_TO_LANG_OTHR, (const void**)&D.p2l_othr, nullptr, 2},
      {CLDT_ULSCRIPT_RTYPE, (const void**)&D.rtype, &D.n_scripts, 1},
      {CLDT_ULSCRIPT_DEFAULT_LANG, (const void**)&D.deflang, nullptr, 2},
      {CLDT_CLOSEST_ALT, (const void**)&D.closest, &D.n_closest, 2},
      {CLDT_CLOSE_SET, (const void**)&D.close_set, &D.n_langs, 1},
  };
  for (auto& s : secs) {
    if (!section(t->blob, s.id, &off, &size)) return CLD_EINVAL;
    *s.dst = at<const void*>(off);
    if (s.count) *s.count = (uint32_t)(size / s.elem);
  }
  {  // fixed-size maps indexed by a byte (per-script numbers, kLgProbV2Tbl rows) or by script
    auto sz = [&](uint32_t id) { uint64_t z = 0; section(t->blob, id, nullptr, &z); return z; };
    if (sz(CLDT_PLANG_TO_LANG_LATN) < 512 || sz(CLDT_PLANG_TO_LANG_OTHR) < 512 || sz(CLDT_LGPROB) < 240 * 8 ||
        sz(CLDT_ULSCRIPT_DEFAULT_LANG) < 2ull * D.n_scripts || D.n_scripts == 0 || D.n_langs == 0)
      return CLD_EINVAL;
  }
  {  // the wavefront kernel's packed tote relies on small score bytes (kMaxLgProbScore)
    if (!section(t->blob, CLDT_LGPROB, &off, &size) || size % 8 || off % 4) return CLD_EINVAL;
    for (uint64_t r = 0; r < size; r += 8)
      for (int k = 5; k < 8; ++k)
        if (t->blob[off + r + k] > kMaxLgProbScore) {
          fprintf(stderr, "cld_mi355x: kLgProbV2Tbl score %d exceeds %d\n", t->blob[off + r + k], kMaxLgProbScore);
          return CLD_EINVAL;
        }
  }
  const cldt_meta& M = t->meta;
  D.latin = M.ulscript_latin; D.cyrillic = M.ulscript_cyrillic; D.arabic = M.ulscript_arabic;
  D.common = M.ulscript_common; D.inherited = M.ulscript_inherited;
  D.unknown_lang = M.unknown_language; D.english = M.english; D.tg_unknown = M.tg_unknown_language;
  D.french = M.french; D.italian = M.italian; D.german = M.german; D.spanish = M.spanish;
  D.hawaiian = M.hawaiian;
  t->codes.clear();
  t->names.clear();
  for (const std::string& c : strings(t->blob, CLDT_LANG_CODES)) t->codes.push_back(intern(c));
  for (const std::string& c : strings(t->blob, CLDT_LANG_NAMES)) t->names.push_back(intern(c));
  {  // optional HTML-mode sections: entity names (a sorted string table), their
     // code points, the cp1252 fix-up; all three or none
    uint64_t no = 0, ns = 0, vo = 0, vs = 0, co = 0, cs = 0;
    const uint8_t* np = section(t->blob, CLDT_ENTITY_NAMES, &no, &ns);
    const uint8_t* vp = section(t->blob, CLDT_ENTITY_VALUES, &vo, &vs);
    const uint8_t* cp = section(t->blob, CLDT_CP1252_FIX, &co, &cs);
    D.ent_names = nullptr; D.ent_values = nullptr; D.cp1252 = nullptr; D.n_ent = 0;
    if (np && vp && cp) {
      const std::vector<std::string> ent = strings(t->blob, CLDT_ENTITY_NAMES);
      if (ent.empty() || ent.size() * 4 != vs || cs < 256 * 4 || ns < 4ull * (ent.size() + 2)) return CLD_EINVAL;
      for (const std::string& e : ent)            // the device compares names NUL-terminated
        if (e.size() >= 16) return CLD_EINVAL;
      D.ent_names = at<const uint8_t*>(no);
      D.ent_values = at<const int32_t*>(vo);
      D.cp1252 = at<const uint32_t*>(co);
      D.n_ent = (uint32_t)ent.size();
    }
  }
  {  // optional hint sections (host only)
    cld::HintView& h = t->hints;
    h = cld::HintView();
    auto tbl = [&](uint32_t id) -> const uint8_t* {   // cldt_hint_entry table + pool, checked
      uint64_t z = 0;
      const uint8_t* p = section(t->blob, id, nullptr, &z);
      if (!p || z < 4) return nullptr;
      const uint32_t n = *(const uint32_t*)p;
      if (4ull + (uint64_t)n * sizeof(cldt_hint_entry) > z) return nullptr;
      const cldt_hint_entry* e = (const cldt_hint_entry*)(p + 4);
      const uint64_t pool = z - 4 - (uint64_t)n * sizeof(cldt_hint_entry);
      const char* ps = (const char*)(e + n);
      for (uint32_t i = 0; i < n; ++i) {
        if (e[i].key_off >= pool || !memchr(ps + e[i].key_off, 0, pool - e[i].key_off)) return nullptr;
        if (e[i].code_off != 0xFFFFFFFFu &&
            (e[i].code_off >= pool || !memchr(ps + e[i].code_off, 0, pool - e[i].code_off)))
          return nullptr;
      }
      return p;
    };
    uint64_t az = 0, rz = 0, ez = 0;
    const uint8_t* act = section(t->blob, CLDT_HINT_CODE_ACTION, nullptr, &az);
    const uint8_t* rem = section(t->blob, CLDT_HINT_CODE_REMAP, nullptr, &rz);
    const uint8_t* enc = section(t->blob, CLDT_HINT_ENCODING, nullptr, &ez);
    if (act && rem && enc && az >= 256 && rz >= 256) {
      h.langtag1 = tbl(CLDT_HINT_LANGTAG1);
      h.langtag2 = tbl(CLDT_HINT_LANGTAG2);
      h.tld = tbl(CLDT_HINT_TLD);
      h.action = act; h.remap = rem;
      h.enc = (const int16_t*)enc; h.n_enc = (uint32_t)(ez / 2);
      const uint8_t* b = t->blob.data();
      h.l2p = b + (uintptr_t)D.l2p; h.l2p_size = D.l2p_size;
      h.p2l_latn = (const uint16_t*)(b + (uintptr_t)D.p2l_latn);
      h.p2l_othr = (const uint16_t*)(b + (uintptr_t)D.p2l_othr);
      h.close_set = b + (uintptr_t)D.close_set; h.n_langs = D.n_langs;
      h.unknown_language = t->meta.unknown_language;
      h.chinese = h.chinese_t = 0xFFFFFFFFu;
      for (size_t i = 0; i < t->codes.size(); ++i) {
        if (strcmp(t->codes[i], "zh") == 0) h.chinese = (uint32_t)i;
        if (strcmp(t->codes[i], "zh-Hant") == 0) h.chinese_t = (uint32_t)i;
      }
      if (!h.ok()) h = cld::HintView();
    }
  }
  const cldt_table_header* q = (const cldt_table_header*)section(t->blob, CLDT_QUAD, nullptr, nullptr);
  // which quadgram table is live: the empty placeholder (Q0, what the reference
  // itself can run without the missing quadchrome blob), the synthetic Q1 test
  // table, or one imported from a cld2 data file / other CLDT
  std::string quad = "other";
  uint64_t psize = 0;
  const uint8_t* prov = section(t->blob, CLDT_PROVENANCE, nullptr, &psize);
  const std::string pv = prov ? std::string((const char*)prov, psize) : std::string();
  if (D.quad.n_buckets <= 1 && D.quad.n_ind <= 1 && D.quad2.size == 0) quad = "empty-Q0";
  else if (pv.find("SYNTHETIC") != std::string::npos) quad = "synthetic-Q1";
  t->version = "cld-mi355x 2.0 tables=" + label + " quad=" + quad + " quad_build=" + std::to_string(q->build_date);
  return CLD_OK;
}

int load_tables(const char* path, HostTables* t) {
  int rc = read_file(path, &t->blob);
  if (rc) { fprintf(stderr, "cld_mi355x: cannot read tables %s\n", path); return CLD_EINVAL; }
  return parse_tables(t, path);
}

template <class P>
P rebase(P off, const uint8_t* base) {
  return reinterpret_cast<P>(const_cast<uint8_t*>(base) + (uintptr_t)off);
}

DevTables device_tables(const DevTables& o, const uint8_t* d) {
  DevTables T = o;
  auto sm = [&](DevSM& s) {
    if (s.t8) s.t8 = rebase(s.t8, d);
    if (s.t16) s.t16 = rebase(s.t16, d);
    s.remap = rebase(s.remap, d); s.rstr = rebase(s.rstr, d);
  };
  sm(T.script); sm(T.lower); sm(T.scan); sm(T.uni);
  for (DevTbl* t : {&T.compat, &T.deltabi, &T.distinctbi, &T.quad, &T.quad2, &T.deltaocta, &T.distinctocta}) {
    t->b = rebase(t->b, d); t->ind = rebase(t->ind, d);
  }
  T.expected = rebase(T.expected, d); T.lgprob = rebase(T.lgprob, d); T.l2p = rebase(T.l2p, d);
  T.p2l_latn = rebase(T.p2l_latn, d); T.p2l_othr = rebase(T.p2l_othr, d); T.rtype = rebase(T.rtype, d);
  T.deflang = rebase(T.deflang, d); T.closest = rebase(T.closest, d); T.close_set = rebase(T.close_set, d);
  if (T.ent_names) {
    T.ent_names = rebase(T.ent_names, d); T.ent_values = rebase(T.ent_values, d); T.cp1252 = rebase(T.cp1252, d);
  }
  return T;
}

// ------------------------------------------------------------ per-GPU context
// Request-sized batches of short documents (run_tiny): at most kTinyDocs
// documents of at most kWaveCap bytes.  One pinned block and its device twin
// per tiny slot, laid out so that one upload and one download carry a call:
//   [results (n x 40 B, ending at kTinyCtrOff) | (unused) | offsets | text]
constexpr size_t kTinyDocs = 1024;
constexpr size_t kTinyCtrOff = kTinyDocs * sizeof(cld_result);
constexpr size_t kTinyOffsOff = kTinyCtrOff + kCtrSlots * sizeof(uint32_t);
constexpr size_t kTinyBlock = kTinyOffsOff + (kTinyDocs + 1) * sizeof(uint64_t) + kTinyDocs * kWaveCap + 256;
constexpr int kTinySlotsMax = 4;   // calls in flight per context (each its own stream); CLD_TINY_SLOTS, default 4
int tiny_slots() {
  static const int v = getenv("CLD_TINY_SLOTS") ? std::max(1, std::min(kTinySlotsMax, atoi(getenv("CLD_TINY_SLOTS")))) : 4;
  return v;
}
struct TinySlot {
  hipStream_t s = nullptr;
  uint8_t* h = nullptr;          // pinned
  uint8_t* hd = nullptr;         // the pinned block's device address (zero-copy mode)
  uint8_t* dv = nullptr;         // device
  uint32_t* d_rq = nullptr;      // k_wave's re-queue list
  std::mutex mu;
};

struct Device {
  int id = 0;
  hipStream_t stream = nullptr;
  uint8_t* d_blob = nullptr;
  DevTables T{};
  DevTables* d_T = nullptr;   // T in HBM (k_long reads the table set through a pointer)
  uint8_t* d_arena = nullptr;
  uint64_t stride = 0;
  int lanes = 0;
  uint8_t* d_slots = nullptr; // k_long per-wave slots 
  cld_result* d_spec_out = nullptr;   // k_long's speculative pass-2 results (small batches; CLD_LONG_SPEC=0: off)
  uint32_t* d_spec_take = nullptr;
  int n_slots = 0;               // the fused k_long's resident waves (its grid)
  // Staged long-document path (cld_launch_staged; CLD_LONG_STAGED=0: off):
  // pass 1's spans of every long document in a store (CLD_LONG_STORE_MB, 8 GB
  // default; a document finding it full takes the fused kernel), the list
  // entries' regions (meta) and the stage lists
  bool staged = false;
  int st_waves = 0;             // slots the staged kernels use (>= n_slots slots are allocated)
  uint8_t* d_store = nullptr; uint64_t store_bytes = 0;
  uint64_t* d_meta = nullptr; size_t meta_cap = 0;
  uint32_t* d_stlists = nullptr; size_t stlists_cap = 0;   // ok / pass-2 / fallback lists, 3 x cap
  uint32_t* d_parlists = nullptr; size_t parlists_cap = 0; // span-parallel: 2 document lists + 2 group lists
  uint32_t* d_requeue2 = nullptr;
  size_t requeue2_cap = 0;
  bool long_order = true;       // k_long takes its list longest first (CLD_LONG_ORDER=0: arrival order)
  uint32_t* d_lsorted = nullptr; size_t lsorted_cap = 0;   // k_long list, longest first
  uint8_t* d_lkey = nullptr; size_t lkey_cap = 0;          // length bucket per re-queued document
  uint32_t* d_lhist = nullptr;                             // bucket histogram + scatter cursors
  uint32_t* h_trace = nullptr;  // CLD_TRACE=1: pinned host progress words, 4 per k_long wave
  uint32_t* d_dbg = nullptr;    // CLD_DEBUG_DOC=i: k_long dumps document i's rounds/chunks
  uint32_t dbg_doc = 0xFFFFFFFFu;
  uint32_t fault_doc = 0xFFFFFFFFu;   // CLD_FAULT_DOC=i (tests): batch document i gets no result in k_long
  double trace_timeout = 0;
  unsigned long long* d_prof = nullptr;   // per-stage cycle sums (CLD_PROFILE_STAGES=1)
  uint32_t* d_counters = nullptr;
  uint32_t* d_requeue = nullptr;
  size_t requeue_cap = 0;
  uint8_t* d_buf = nullptr; size_t buf_cap = 0;
  uint64_t* d_offs = nullptr; size_t offs_cap = 0;
  cld_result* d_out = nullptr; size_t out_cap = 0;
  uint8_t* d_sbuf = nullptr; size_t sbuf_cap = 0;        // prepared text (CLD_FLAG_STRIP_EXTRAS / CSTRING)
  uint8_t* d_hbuf = nullptr; size_t hbuf_cap = 0;        // HTML pages rewritten into plain text (cld_html.hip)
  uint8_t* d_hflag = nullptr; size_t hflag_cap = 0;      //   and their entity lookahead marks
  uint32_t* d_hpos = nullptr; size_t hpos_cap = 0;       //   and (vec mode) each byte's page offset
  uint64_t* d_soffs = nullptr; size_t soffs_cap = 0;
  uint8_t* d_sscr = nullptr; size_t sscr_cap = 0;
  hipEvent_t ev[4]{};
  std::vector<std::array<hipEvent_t, 4>> ev_pool;   // one set per enqueue since reset
  size_t ev_used = 0;
  cld_batch_stats last{};
  uint64_t last_n = 0;
  bool stats_pending = false;
  // Every batch on this device reuses the scratch above (counters, re-queue
  // lists, k_long slots, staging).  `done` is recorded after a batch's last
  // launch and every enqueue makes its stream wait on it first, so batches on
  // different caller streams (or the runtime's own) execute one after another.
  hipEvent_t done = nullptr;
  // Streamed host path (run_host_shard): two chunk slots, each with pinned
  // staging and device buffers; uploads, kernels and downloads on three
  // streams so chunk k+1's upload and chunk k-1's download overlap chunk k.
  struct Slot {
    uint8_t* h_in = nullptr; size_t h_in_cap = 0;        // pinned: document bytes
    uint64_t* h_offs = nullptr; size_t h_offs_cap = 0;   // pinned: offsets (caller's, not rebased)
    cld_result* h_out = nullptr; size_t h_out_cap = 0;   // pinned: results
    uint8_t* d_in = nullptr; size_t d_in_cap = 0;
    uint64_t* d_offs = nullptr; size_t d_offs_cap = 0;
    cld_result* d_out = nullptr; size_t d_out_cap = 0;
    uint8_t* h_sp = nullptr; size_t h_sp_cap = 0;        // cld_detect_batch_ex: routing bits + priors
    uint32_t* h_pri = nullptr; size_t h_pri_cap = 0;
    uint8_t* d_sp = nullptr; size_t d_sp_cap = 0;
    uint32_t* d_pri = nullptr; size_t d_pri_cap = 0;
    hipEvent_t up = nullptr, comp = nullptr, down = nullptr;
    size_t pending_n = 0; cld_result* pending_dst = nullptr;   // results to hand over once `down` fires
    bool busy = false;
  } hs[2];
  hipStream_t up_stream = nullptr, down_stream = nullptr;
  uint32_t* h_ctr = nullptr;        // pinned: per-chunk counter snapshots (kCtrSlots each)
  size_t h_ctr_cap = 0;
  uint32_t* d_ctrs = nullptr;       // device: per-chunk counters of one streamed call (kCtrSlots each)
  size_t ctrs_cap = 0;
  // ResultChunkVector mode (cld_detect_batch_vec): its own lane arena, made on first use
  struct Vec {
    uint8_t* arena = nullptr; uint64_t stride = 0; int lanes = 0;
    uint8_t* in = nullptr; size_t in_cap = 0;
    uint64_t* offs = nullptr; size_t offs_cap = 0;
    cld_result* out = nullptr; size_t out_cap = 0;
    uint8_t* sp = nullptr; size_t sp_cap = 0;
    uint32_t* pri = nullptr; size_t pri_cap = 0;
    cld_chunk* pool = nullptr; size_t pool_cap = 0;
    uint64_t* pool_off = nullptr; size_t pool_off_cap = 0;
    int32_t* nch = nullptr; size_t nch_cap = 0;
    uint64_t* pos = nullptr; size_t pos_cap = 0;
    uint32_t* order = nullptr; size_t order_cap = 0;
    cld_chunk* compact = nullptr; size_t compact_cap = 0;
    uint8_t* vslots = nullptr;   // k_long<VEC>: one VecSlot per slot of d_slots (on first use)
  } vec;
  TinySlot tiny[kTinySlotsMax];   // run_tiny: k_wave-only calls, independent of the scratch above (tiny_slots() used)
  std::atomic<unsigned> tiny_rr{0};
  std::mutex mu;
  std::atomic<int> inflight{0};   // calls routed to this context and not yet returned (pick_context)
};

std::mutex g_init_mu;
// Table generation lock: every batch call holds it shared from its host-side
// ApplyHints through its last kernel, a table swap (cld_load_data_*,
// cld_unload_data) holds it exclusively.  So no call reads host tables that
// are being replaced, and a call's priors and device tables come from the
// same table set.  Order: g_init_mu, then g_swap_mu, then a device's mu.
std::shared_mutex g_swap_mu;
bool g_inited = false;
std::atomic<bool> g_ready{false};   // g_inited with g_init_rc == CLD_OK (the lock-free check of every call)
int g_init_rc = CLD_ENODEV;
HostTables g_tab;
std::vector<Device*> g_devs;
bool g_dynamic = false;       // g_tab came from a cld2 dynamic data file (cld_load_data_*)
std::string g_base_path;      // the CLDT the static tables were read from

// The product default is Q0, the empty quadgram table (the reference's own
// placeholder pattern): out of the box no answer comes from fabricated quad
// data.  Tests and the benchmark opt into the synthetic Q1 table explicitly
// (CLD_MI355X_TABLES), and a real table arrives through cld_load_data_*.
std::string default_tables_path() {
  if (const char* e = getenv("CLD_MI355X_TABLES")) return e;
  Dl_info info;
  if (dladdr((void*)&default_tables_path, &info) && info.dli_fname) {
    std::string so = info.dli_fname;
    std::string dir = so.substr(0, so.find_last_of('/'));
    return dir + "/../data/cld2_q0.cldt";
  }
  return "language-detector_amd/data/cld2_q0.cldt";
}

template <class T>
int grow(T** p, size_t* cap, size_t need) {
  if (*cap >= need) return CLD_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  size_t n = std::max(need, *cap * 3 / 2);
  if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) { *cap = 0; return CLD_ENOMEM; }
  *cap = n;
  return CLD_OK;
}

// Table blob -> HBM (once per GPU, and again when dynamic data replaces the
// tables), in two steps so a multi-GPU swap is all-or-nothing: stage_tables
// allocates and fills a new copy (the old one stays live), then commit_tables
// drains the device and swaps it in, or discard_tables frees it.
struct StagedTables {
  uint8_t* blob = nullptr;
  uint64_t* cpt = nullptr;
  uint64_t* keytab = nullptr;
  uint64_t* adds = nullptr;
  DevTables T{};
};

int stage_tables(Device* d, const HostTables& t, StagedTables* st) {
  HIP_OK(hipSetDevice(d->id));
  HIP_OK(hipMalloc(&st->blob, t.blob.size()));
  HIP_OK(hipMemcpy(st->blob, t.blob.data(), t.blob.size(), hipMemcpyHostToDevice));
  st->T = device_tables(t.offs, st->blob);
  // per-character property table for the long-document kernel, built from the uploaded machines
  HIP_OK(hipMalloc(&st->cpt, cld_cpt_entries() * sizeof(uint64_t)));
  HIP_OK(cld_build_cpt(&st->T, st->cpt, d->stream));
  HIP_OK(hipMalloc(&st->keytab, cld_keytab_entries() * sizeof(uint64_t)));
  HIP_OK(cld_build_keytab(&st->T, st->keytab, d->stream));
  HIP_OK(hipMalloc(&st->adds, std::max<size_t>(cld_adds_entries(&st->T), 1) * sizeof(uint64_t)));
  HIP_OK(cld_build_adds(&st->T, st->adds, d->stream));   // sets T.<table>.adds (compat.adds is the base)
  HIP_OK(hipStreamSynchronize(d->stream));
  st->T.cpt = st->cpt;
  st->T.keytab = st->keytab;
  return CLD_OK;
}

void discard_tables(Device* d, StagedTables* st) {
  (void)hipSetDevice(d->id);
  if (st->blob) (void)hipFree(st->blob);
  if (st->cpt) (void)hipFree(st->cpt);
  if (st->keytab) (void)hipFree(st->keytab);
  if (st->adds) (void)hipFree(st->adds);
  *st = StagedTables();
}

// The caller holds d->mu or owns d exclusively.
int commit_tables(Device* d, StagedTables* st) {
  HIP_OK(hipSetDevice(d->id));
  HIP_OK(hipDeviceSynchronize());   // batches enqueued on caller streams may still read the old blob
  if (d->d_blob) (void)hipFree(d->d_blob);
  if (d->T.cpt) (void)hipFree((void*)d->T.cpt);
  if (d->T.keytab) (void)hipFree((void*)d->T.keytab);
  if (d->T.compat.adds) (void)hipFree((void*)d->T.compat.adds);
  d->d_blob = st->blob;
  d->T = st->T;
  *st = StagedTables();
  if (!d->d_T) HIP_OK(hipMalloc(&d->d_T, sizeof(DevTables)));
  HIP_OK(hipMemcpy(d->d_T, &d->T, sizeof(DevTables), hipMemcpyHostToDevice));
  return CLD_OK;
}

int upload_tables(Device* d, const HostTables& t) {
  StagedTables st;
  int rc = stage_tables(d, t, &st);
  if (rc) { discard_tables(d, &st); return rc; }
  return commit_tables(d, &st);
}

// Replace the tables on every initialised GPU, or on none.  Caller holds g_init_mu.
int swap_tables_all(const HostTables& nt);

int init_device(Device* d) {
  HIP_OK(hipSetDevice(d->id));
  // CLD_SYNC=block|spin|yield: how host threads wait for the GPU (HIP's
  // default decides by itself).  Waiting callers burn CPU when they spin,
  // which a CPU-quota'd service may not have to spare.
  if (const char* e = getenv("CLD_SYNC")) {
    const unsigned f = !strcmp(e, "block") ? hipDeviceScheduleBlockingSync
                       : !strcmp(e, "spin") ? hipDeviceScheduleSpin
                       : !strcmp(e, "yield") ? hipDeviceScheduleYield : hipDeviceScheduleAuto;
    (void)hipSetDeviceFlags(f);
    (void)hipGetLastError();
  }
  HIP_OK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&d->up_stream, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&d->down_stream, hipStreamNonBlocking));
  HIP_OK(hipEventCreateWithFlags(&d->done, hipEventDisableTiming));
  HIP_OK(hipEventRecord(d->done, d->stream));
  for (auto& h : d->hs) {
    HIP_OK(hipEventCreateWithFlags(&h.up, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&h.comp, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&h.down, hipEventDisableTiming));
  }
  if (int rc = upload_tables(d, g_tab)) return rc;
  for (int k = 0; k < tiny_slots(); ++k) {
    TinySlot& t = d->tiny[k];
    HIP_OK(hipStreamCreateWithFlags(&t.s, hipStreamNonBlocking));
    HIP_OK(hipHostMalloc((void**)&t.h, kTinyBlock, hipHostMallocDefault));
    HIP_OK(hipHostGetDevicePointer((void**)&t.hd, t.h, 0));
    HIP_OK(hipMalloc(&t.dv, kTinyBlock));
    HIP_OK(hipMalloc(&t.d_rq, kTinyDocs * sizeof(uint32_t)));
  }
  HIP_OK(hipMalloc(&d->d_counters, kCtrSlots * sizeof(uint32_t)));
  HIP_OK(hipMalloc(&d->d_lhist, 256 * sizeof(uint32_t)));
  if (const char* e = getenv("CLD_LONG_ORDER")) d->long_order = atoi(e) != 0;
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, d->id));
  if (const char* e = getenv("CLD_PROFILE_STAGES")) {
    if (atoi(e) > 0) {
      HIP_OK(hipMalloc(&d->d_prof, 16 * sizeof(unsigned long long)));
      HIP_OK(hipMemset(d->d_prof, 0, 16 * sizeof(unsigned long long)));
    }
  }
  // k_long: one slot per resident wavefront of its persistent grid; every
  // document longer than k_wave takes, or that k_wave hands on, runs there
  int waves = 4 * cld_long_waves_per_simd();   // fill every SIMD at the kernel's occupancy
  if (const char* e = getenv("CLD_LONG_WAVES")) waves = std::max(1, atoi(e));
  int n_slots = (prop.multiProcessorCount * waves / kLongWPB) * kLongWPB;
  const uint64_t slot = cld_long_slot_bytes();
  while (n_slots > kLongWPB && (uint64_t)n_slots * slot > (8ull << 30)) n_slots -= kLongWPB;
  if (n_slots < kLongWPB) return CLD_ENOMEM;
  int alloc_slots = n_slots;
  if (n_slots > 0 && !(getenv("CLD_LONG_STAGED") && atoi(getenv("CLD_LONG_STAGED")) == 0)) {
    const int st = prop.multiProcessorCount * 4 * cld_staged_waves_per_simd();
    uint64_t mb = 8192;
    if (const char* e = getenv("CLD_LONG_STORE_MB")) mb = strtoull(e, nullptr, 10);
    // (64 KB past the last region: the span readers' slack reads stay inside the allocation)
    if (mb && (uint64_t)st * slot <= (12ull << 30) && hipMalloc(&d->d_store, (mb << 20) + (64u << 10)) == hipSuccess) {
      d->store_bytes = mb << 20;
      d->st_waves = st;
      d->staged = true;
      alloc_slots = std::max(n_slots, st);
    } else {
      (void)hipGetLastError();
      d->d_store = nullptr;
    }
  }
  if (n_slots > 0) {
    HIP_OK(hipMalloc(&d->d_slots, (uint64_t)alloc_slots * slot));
    HIP_OK(hipMemset(d->d_slots, 0, (uint64_t)alloc_slots * slot));   // predictor epochs start at 0
    d->n_slots = n_slots;
    const char* sp = getenv("CLD_LONG_SPEC");
    if (!sp || atoi(sp) != 0) {
      const size_t m = std::max<size_t>(1, cld_long_spec_docs(n_slots));
      HIP_OK(hipMalloc(&d->d_spec_out, m * sizeof(cld_result)));
      HIP_OK(hipMalloc(&d->d_spec_take, m * sizeof(uint32_t)));
    }
  }
  if (const char* e = getenv("CLD_FAULT_DOC")) d->fault_doc = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("CLD_DEBUG_DOC")) {
    d->dbg_doc = (uint32_t)atoll(e);
    HIP_OK(hipMalloc(&d->d_dbg, 64u << 20));
  }
  if (const char* e = getenv("CLD_TRACE")) {
    if (atoi(e) > 0 && n_slots > 0) {
      HIP_OK(hipHostMalloc((void**)&d->h_trace, (size_t)n_slots * 16, hipHostMallocCoherent | hipHostMallocMapped));
      memset(d->h_trace, 0xFF, (size_t)n_slots * 16);
      d->trace_timeout = 20.0;
      if (const char* t = getenv("CLD_TRACE_TIMEOUT")) d->trace_timeout = atof(t);
    }
  }
  return CLD_OK;
}

constexpr uint32_t kPrepFlags = CLD_FLAG_STRIP_EXTRAS | CLD_FLAG_CSTRING;
// the reference's public flags the kernels apply; its debug-output flags are accepted and ignored
constexpr uint32_t kCldFlags = CLD_FLAG_SCORE_AS_QUADS | CLD_FLAG_BEST_EFFORT;
constexpr uint32_t kPublicFlags = kCldFlags | CLD_FLAG_DEBUG_MASK;

// A long list this short goes whole to the fused k_long, whose two-wave
// speculation halves a lone long document's latency: 64 documents, or
// CLD_LONG_SMALL documents (0: the staged path for every batch).  Up to
// round 5 the bound was 4 per fused wave (16K documents); request-sized
// batches (~1,000 C5 documents, ~200 of them long) run better staged, where
// span-parallel scoring splits their many-span pages: 1 caller 96.6K ->
// 106K docs/s (p99 34 -> 17 ms), 32 callers 699K -> 875K
// (profiles/round5_req_staged_ab.jsonl).
uint32_t small_long_list(const Device* d) {
  (void)d;
  static const long v = getenv("CLD_LONG_SMALL") ? atol(getenv("CLD_LONG_SMALL")) : -1;
  return v >= 0 ? (uint32_t)v : 64u;
}
// ...unless it holds a document of CLD_LONG_SMALL_KB KB or more (default 0:
// no such rule).  A page that long may hold thousands of spans, which one
// fused wave scores in tens of milliseconds (a 64 KB page of 3,082 spans:
// 44-48 ms) where the staged path splits them into span-parallel groups.
// detect_language on C5 documents (profiles/round6_dl_rate_c5_heavy_ab.jsonl),
// 32 KB against off: the slowest call 45-48 -> 24-29 ms, p99 at 64 callers
// 20 -> 17 ms, but 8 callers 11.3K -> 10.8K docs/s (the few-span 32-64 KB
// pages lose the fused kernel's two-wave speculation) -- a tail-latency
// option, not the default.
uint64_t small_list_heavy_bytes() {
  static const long v = getenv("CLD_LONG_SMALL_KB") ? atol(getenv("CLD_LONG_SMALL_KB")) : 0;
  return v > 0 ? (uint64_t)v << 10 : ~0ull;
}

// Batches holding a document of this many KB go to the fused k_long whole
// (CLD_LONG_HEAVY_KB; default 0: never).  Before span-parallel scoring a C5
// batch's many-span 64 KB pages (~48 ms on one wave) repeated their latency
// in every stage kernel, and 20 KB kept C5 on the fused kernel (18.1M
// docs/s); with it the staged path runs C5 at 22.0M (gpurun_out/r5r).
uint32_t heavy_kb() {
  static const uint32_t v = getenv("CLD_LONG_HEAVY_KB") ? (uint32_t)atoi(getenv("CLD_LONG_HEAVY_KB")) : 0u;
  return v;
}

// Text preparation (handlers.go:150-151) on device d: documents [buf, offs) ->
// prepared documents in d->d_sbuf / d->d_soffs.  cap_bytes bounds offs[n].
int enqueue_prepare(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, uint64_t cap_bytes,
                    uint32_t flags, hipStream_t s) {
  HIP_OK(hipStreamWaitEvent(s, d->done, 0));   // the previous batch may still read d_sbuf
  if (grow(&d->d_sbuf, &d->sbuf_cap, std::max<size_t>(cap_bytes + n, 1))) return CLD_ENOMEM;
  if (grow(&d->d_soffs, &d->soffs_cap, n + 1)) return CLD_ENOMEM;
  if (grow(&d->d_sscr, &d->sscr_cap, cld_strip_scratch_bytes((int)n))) return CLD_ENOMEM;
  HIP_OK(cld_launch_strip_offsets(buf, offs, (int)n, flags & kPrepFlags, d->d_soffs, d->d_sscr, s));
  HIP_OK(cld_launch_strip_write(buf, offs, (int)n, flags & kPrepFlags, d->d_soffs, d->d_sbuf, s));
  return CLD_OK;
}

// Enqueue the whole pipeline for n documents already on device d.  special /
// priors (device, nullable): cld_detect_batch_ex's per-document routing bits
// and ApplyHints langprobs (16 per document); HTML documents skip the wave and
// wave kernel and run in k_long (rewritten, or on its sequential span source),
// hinted plain ones take the wave / long kernels with their priors.  cflags: CLD2's public flags (kCldFlags).
// html_bytes > 0 (the batch holds HTML pages, special & kSpecialHtml; special
// is then the runtime's own device copy): the pages are first rewritten into
// plain text (cld_html.hip, k_html_rewrite) in d_hbuf, indexed like buf, whose
// document bytes span [html_base, html_base + html_bytes) of the offsets.
int enqueue(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out, hipStream_t s,
            const uint8_t* special = nullptr, const uint32_t* priors = nullptr, uint32_t cflags = 0,
            uint64_t html_base = 0, uint64_t html_bytes = 0, uint32_t* ctr = nullptr, int64_t long_hint = -1) {
  cflags &= kCldFlags;
  const uint8_t *hbuf = nullptr, *hflag = nullptr;
  uint32_t *hpos = nullptr, *hgap = nullptr;
  if (special && html_bytes) {
    if (grow(&d->d_hbuf, &d->hbuf_cap, html_bytes) || grow(&d->d_hflag, &d->hflag_cap, html_bytes)) return CLD_ENOMEM;
    hbuf = d->d_hbuf - html_base;
    hflag = d->d_hflag - html_base;
    // pages of kMaxScriptBytes and more also get each rewritten byte's page
    // offset: their span soft limit reads the raw bytes left
    if (html_bytes >= (uint64_t)kHtmlSoftMin) {
      if (grow(&d->d_hpos, &d->hpos_cap, 2 * html_bytes)) return CLD_ENOMEM;
      hpos = d->d_hpos - html_base;
      hgap = d->d_hpos + html_bytes - html_base;
    }
  }
  if (grow(&d->d_requeue, &d->requeue_cap, std::max<size_t>(n, 1))) return CLD_ENOMEM;
  if (grow(&d->d_requeue2, &d->requeue2_cap, std::max<size_t>(n, 1))) return CLD_ENOMEM;
  if (d->n_slots > 0 && d->long_order) {
    if (grow(&d->d_lsorted, &d->lsorted_cap, std::max<size_t>(n, 1))) return CLD_ENOMEM;
    if (grow(&d->d_lkey, &d->lkey_cap, std::max<size_t>(n, 1))) return CLD_ENOMEM;
  }
  if (d->ev_used == d->ev_pool.size()) {
    std::array<hipEvent_t, 4> t{};
    for (auto& e : t) HIP_OK(hipEventCreate(&e));
    d->ev_pool.push_back(t);
  }
  auto& ev = d->ev_pool[d->ev_used++];
  HIP_OK(hipStreamWaitEvent(s, d->done, 0));   // serialise with the previous batch's scratch use
  // counters: the device's own (zeroed here), or the caller's region (ctr,
  // kCtrSlots words, zeroed by the caller: the streamed host path zeroes one
  // region per chunk in a single memset and reads them back in one copy)
  if (!ctr) {
    ctr = d->d_counters;
    HIP_OK(hipMemsetAsync(ctr, 0, kCtrSlots * sizeof(uint32_t), s));
  }
  if (d->d_dbg) HIP_OK(hipMemsetAsync(d->d_dbg, 0, 4, s));
  HIP_OK(hipEventRecord(ev[0], s));
  if (hbuf)
    HIP_OK(cld_launch_html_rewrite(d->d_T, buf, offs, (int)n, const_cast<uint8_t*>(special), const_cast<uint8_t*>(hbuf),
                                   const_cast<uint8_t*>(hflag), hpos, hgap, kHtmlSoftMin,
                                   d->d_prof ? d->d_prof + 7 : nullptr, s));
  // HTML pages the rewrite did not take join k_long's list (its sequential
  // span source scans them in HTML mode, cld_seq.hip)
  HIP_OK(cld_launch_wave(&d->T, buf, offs, (int)n, out, d->d_requeue, ctr, d->d_prof, special, d->d_requeue,
                         kCtrRequeue, cflags, priors, hbuf, hflag, d->long_order ? d->d_lhist : nullptr, s));
  HIP_OK(hipEventRecord(ev[1], s));
  {
    const uint32_t* list = d->d_requeue;
    if (d->long_order) {
      HIP_OK(cld_launch_order_long(offs, d->d_requeue, ctr, d->d_lkey, d->d_lhist, d->d_lsorted, n > 0, s));
      list = d->d_lsorted;
    }
    // the staged path takes the list unless diagnostics (the fused kernel's
    // trace / debug dump / stage cycles) are on; what it does not take goes to
    // the fused kernel as the fallback list
    // long_hint (the host path, which holds the offsets): documents longer
    // than k_wave takes.  A list that short goes whole to the fused kernel
    // anyway, so the eight staged launches are skipped (each costs its
    // dispatch even when its list is empty: ~60 us per chunk of tweets)
    const bool staged = d->staged && !d->h_trace && !d->d_dbg && !d->d_prof &&
                        !(long_hint >= 0 && small_long_list(d) > 0 && long_hint <= (int64_t)small_long_list(d));
    int ctr_total = kCtrRequeue, ctr_deq = kCtrDequeue;
    if (staged) {
      if (grow(&d->d_meta, &d->meta_cap, std::max<size_t>(n, 1))) return CLD_ENOMEM;
      if (grow(&d->d_stlists, &d->stlists_cap, 3 * std::max<size_t>(n, 1))) return CLD_ENOMEM;
      const size_t c = d->stlists_cap / 3;
      uint32_t* fall = d->d_stlists + 2 * c;
      // span-parallel lists: documents (n each, passes 1 and 2) and groups
      // (gcap each; a document whose groups find no room takes the fused kernel)
      const size_t np = std::max<size_t>(n, 1), gcap = std::max<size_t>(4 * np, 1u << 16);
      if (grow(&d->d_parlists, &d->parlists_cap, 2 * np + 4 * gcap)) return CLD_ENOMEM;
      // a list of at most small_long_list() documents (64) goes whole to the
      // fused kernel: small batches keep its two-wave speculation (section 6)
      // (the host's count says the list is longer than that, or holds a
      // document of small_list_heavy_bytes() or more: no list goes whole)
      const uint32_t small_total = long_hint > (int64_t)small_long_list(d) ? 0u : small_long_list(d);
      HIP_OK(cld_launch_staged(d->d_T, buf, offs, list, out, d->d_slots, d->st_waves, d->d_store, d->store_bytes,
                               d->d_meta, d->d_stlists, d->d_stlists + c, fall, ctr, cflags, special,
                               priors, hbuf, hflag, hpos, hgap, d->fault_doc, small_total,
                               d->long_order ? d->d_lhist : nullptr, heavy_kb(), d->d_parlists, np, gcap, s));
      list = fall;
      ctr_total = kCtrStFall;
      ctr_deq = kCtrStDqFall;
    }
    HIP_OK(cld_launch_long(d->d_T, buf, offs, list, out, d->d_slots, d->n_slots, d->d_requeue2, ctr, d->h_trace, d->d_dbg, d->dbg_doc,
                           d->d_prof ? d->d_prof + 8 : nullptr, cflags, special, priors, hbuf, hflag, hpos, hgap,
                           d->fault_doc,
                           d->d_spec_out, d->d_spec_take, ctr_total, ctr_deq, ev[2], s));
  }
  HIP_OK(hipEventRecord(ev[3], s));
  HIP_OK(hipEventRecord(d->done, s));
  for (int k = 0; k < 4; ++k) d->ev[k] = ev[k];
  d->last_n = n;
  d->stats_pending = true;
  return CLD_OK;
}

// Adds one batch's device counters to st (docs = documents of that batch).
// short_docs: finished by k_wave; long_docs: by k_long (or the staged path)
// on the parallel span builder; general_docs: by k_long on the sequential
// span source (cld_seq.hip).
void add_counters(Device* d, const uint32_t* c, uint64_t docs, cld_batch_stats* st) {
  (void)d;
  const uint64_t shorts = docs - c[kCtrRequeue];
  st->docs += docs;
  st->general_docs += c[kCtrSeq];
  st->long_docs += c[kCtrRequeue] - c[kCtrSeq];
  st->short_docs += shorts;
  st->passes[0] += shorts + c[kCtrPass1];
  st->passes[1] += c[kCtrPass2];
  st->passes[2] += c[kCtrPass3];
  st->passes[3] += c[kCtrError];
  for (int k = 0; k < 8; ++k) st->long_requeue[k] += c[kCtrWhy + k];
}

int collect_stats(Device* d) {
  if (!d->stats_pending) return CLD_OK;
  uint32_t c[kCtrSlots];
  // the batch may have run on a caller's stream: wait for its last event, then
  // read the counters before any later batch can reset them (the runtime
  // stream waits on `done`, which a later enqueue re-records only after this)
  HIP_OK(hipEventSynchronize(d->ev[3]));
  HIP_OK(hipStreamWaitEvent(d->stream, d->ev[3], 0));
  HIP_OK(hipMemcpyAsync(c, d->d_counters, sizeof(c), hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  float ms1 = 0, ms2 = 0, ms3 = 0;
  HIP_OK(hipEventElapsedTime(&ms1, d->ev[0], d->ev[1]));
  HIP_OK(hipEventElapsedTime(&ms2, d->ev[1], d->ev[2]));
  HIP_OK(hipEventElapsedTime(&ms3, d->ev[2], d->ev[3]));
  cld_batch_stats& st = d->last;
  memset(&st, 0, sizeof(st));
  add_counters(d, c, d->last_n, &st);
  st.short_ms = ms1;
  st.long_ms = ms2;
  st.general_ms = ms3;
  d->stats_pending = false;
  return c[kCtrError] ? CLD_EIO : CLD_OK;
}

// Debug (CLD_TRACE=1): a batch that overruns dumps where every k_long wave is.
// A batch whose stream ends in an error (a faulting kernel) dumps them too.
void watch_trace(Device* d, hipStream_t s) {
  auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) return;
    double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (q == hipErrorNotReady) {
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      if (el <= d->trace_timeout) continue;
      fprintf(stderr, "cld_mi355x: batch still running after %.0f s; k_long waves (doc stage value count):\n", el);
    } else {
      fprintf(stderr, "cld_mi355x: batch failed (%s) after %.3f s; k_long waves (doc stage value count):\n",
              hipGetErrorString(q), el);
    }
    int untouched = 0, exited = 0;
    for (int w = 0; w < d->n_slots; ++w) {
      volatile uint32_t* t = d->h_trace + 4 * w;
      untouched += t[3] == 0xFFFFFFFFu;
      exited += (t[1] & 0xFFFF) == 100;
    }
    fprintf(stderr, "  %d waves: %d never started, %d exited\n", d->n_slots, untouched, exited);
    for (int w = 0; w < d->n_slots; ++w) {
      volatile uint32_t* t = d->h_trace + 4 * w;
      if (t[3] != 0xFFFFFFFFu && ((t[1] & 0xFFFF) != 100 || w < 2))
        fprintf(stderr, "  wave %d: doc %u stage %u (active lanes %u, first %u) value %u count %u\n", w, t[0],
                t[1] & 0xFFFF, (t[1] >> 16) & 0xFF, t[1] >> 24, t[2], t[3]);
    }
    fflush(stderr);
    if (q == hipErrorNotReady) abort();
    return;                                      // (the error reaches the caller at the next sync)
  }
}

// Chunking of the streamed host path: a chunk is at most 64 MB of document
// text and 8K documents per MB (the first three ramp up from 1/8 of that, see
// run_host_shard), so two chunks in flight stay small next to HBM while each
// is still a full-chip launch (C2 host path, pinned buffers, with the ramp:
// 16 MB chunks 7.0 ms, 32 MB 6.3 ms, 64 MB 6.2 ms per 1M documents;
// gpurun_out/r4g).  CLD_CHUNK_MB overrides the byte limit.
uint64_t chunk_bytes() {
  static const uint64_t v = [] {
    uint64_t mb = 64;
    if (const char* e = getenv("CLD_CHUNK_MB")) mb = std::max<uint64_t>(1, strtoull(e, nullptr, 10));
    return mb << 20;
  }();
  return v;
}

bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();   // unregistered pageable memory reports an error: clear it
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

template <class T>
int grow_host(T** p, size_t* cap, size_t need) {
  if (*cap >= need) return CLD_OK;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  size_t n = std::max(need, *cap * 3 / 2);
  if (hipHostMalloc((void**)p, n * sizeof(T), hipHostMallocDefault) != hipSuccess) { *cap = 0; return CLD_ENOMEM; }
  *cap = n;
  return CLD_OK;
}

// Staging copies (pageable caller memory <-> pinned slots) on a persistent
// pool of host threads: one core copies only a few GB/s, and spawning threads
// per chunk cost tens of microseconds each.  The caller takes pieces too; one
// copy runs at a time (they are bandwidth-bound anyway).  CLD_COPY_THREADS
// sets the pool size (default min(16, hardware threads)).
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();        // never destroyed: its threads are detached
    return *p;
  }
  void copy(void* dst, const void* src, size_t n) {
    constexpr size_t kPiece = 2u << 20;
    Job j{(uint8_t*)dst, (const uint8_t*)src, n, kPiece, (n + kPiece - 1) / kPiece};
    if (j.pieces <= 1 || workers_ == 0) { memcpy(dst, src, n); return; }
    std::lock_guard<std::mutex> one(job_mu_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      cur_ = &j;
      ++gen_;
    }
    cv_.notify_all();
    const size_t mine = j.run();
    std::unique_lock<std::mutex> lk(mu_);
    j.done += mine;
    cur_ = nullptr;                             // late wakers find no job
    done_cv_.wait(lk, [&] { return j.done == j.pieces && j.refs == 0; });
  }

 private:
  struct Job {
    uint8_t* dst; const uint8_t* src; size_t n, piece, pieces;
    std::atomic<size_t> next{0};
    size_t done = 0; int refs = 0;              // under mu_
    Job(uint8_t* d, const uint8_t* s, size_t n_, size_t p, size_t k) : dst(d), src(s), n(n_), piece(p), pieces(k) {}
    size_t run() {
      size_t k = 0;
      for (size_t i; (i = next.fetch_add(1, std::memory_order_relaxed)) < pieces; ++k) {
        const size_t a = i * piece;
        memcpy(dst + a, src + a, std::min(piece, n - a));
      }
      return k;
    }
  };
  CopyPool() {
    int t = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = getenv("CLD_COPY_THREADS")) t = std::max(1, atoi(e));
    workers_ = t - 1;
    for (int i = 0; i < workers_; ++i) std::thread([this] { work(); }).detach();
  }
  void work() {
    uint64_t seen = 0;
    for (;;) {
      Job* j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (!(j = cur_)) continue;
        ++j->refs;
      }
      const size_t k = j->run();
      std::lock_guard<std::mutex> lk(mu_);
      j->done += k;
      --j->refs;
      done_cv_.notify_all();
    }
  }
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  Job* cur_ = nullptr;
  uint64_t gen_ = 0;
  int workers_ = 0;
};

void par_copy(void* dst, const void* src, size_t n) { CopyPool::get().copy(dst, src, n); }

// Host batch on one device, streamed: documents go in chunks through two
// slots.  Per chunk: stage into pinned memory (skipped when the caller's
// buffers are already pinned), upload on up_stream, the kernels on the
// runtime stream, results back on down_stream.  Offsets are uploaded as the
// caller wrote them and the kernels get `d_in - offs[first]` as their buffer
// base, so no rebasing pass runs anywhere.  Chunk k's staging overlaps chunk
// k-1's kernels; its upload overlaps them too.
// Large pageable batches: the caller's buffers are page-locked for the call
// (hipHostRegister) instead of staged chunk by chunk through pinned copies,
// above CLD_HOST_REGISTER_MB of document text (default 64; 0 = never).
uint64_t register_min_bytes() {
  static const uint64_t v = [] {
    uint64_t mb = 64;
    if (const char* e = getenv("CLD_HOST_REGISTER_MB")) mb = strtoull(e, nullptr, 10);
    return mb ? mb << 20 : ~0ull;
  }();
  return v;
}

// Page-locks [p, p + bytes) for the life of the object when it is not pinned already.
struct HostReg {
  void* p = nullptr;
  bool on = false;
  bool take(const void* q, size_t bytes) {
    if (!bytes) return false;
    if (hipHostRegister(const_cast<void*>(q), bytes, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    p = const_cast<void*>(q);
    on = true;
    return true;
  }
  void release() {
    if (on) (void)hipHostUnregister(p);
    on = false;
  }
  HostReg() = default;
  HostReg(const HostReg&) = delete;
  HostReg& operator=(const HostReg&) = delete;
  ~HostReg() { release(); }
};

// run_host_shard's "some documents failed" return (k_long counted and
// marked them); internal, never returned to a caller.
constexpr int kDocsFailed = 1;

int run_host_stream(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out, uint32_t flags,
                    const uint8_t* special = nullptr, const uint32_t* priors = nullptr, bool html = false) {
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  d->ev_used = 0;
  bool in_pinned = host_pinned(buf + offs[0]) && host_pinned(offs);
  bool out_pinned = host_pinned(out);
  // (declared before any DMA is enqueued: unregistered only after the drain below)
  HostReg reg_buf, reg_offs, reg_out;
  if (offs[n] - offs[0] >= register_min_bytes()) {
    if (!in_pinned) {
      in_pinned = reg_buf.take(buf + offs[0], offs[n] - offs[0]) && reg_offs.take(offs, (n + 1) * sizeof(uint64_t));
      if (!in_pinned) reg_buf.release();
    }
    if (!out_pinned) out_pinned = reg_out.take(out, n * sizeof(cld_result));
  }
  // chunk plan.  The first chunks ramp up (1/8, 1/4, 1/2 of the chunk size):
  // nothing runs until chunk 0 is uploaded, and an upload (~53 GB/s) outruns
  // the kernels (~28 GB/s at C2), so a small first chunk shortens the fill
  // while the next, larger upload still finishes before its kernels are due.
  // A batch whose mean document is longer than k_wave takes is bound by
  // k_long's longest document per launch (one wave scores it start to end),
  // and every chunk pays that tail again: such batches go in chunks four
  // times as large and without the ramp (a coalesced batch of requests is
  // then one launch; C5 requests: 8 callers 193K -> 299K, 64 callers
  // 404K -> 863K docs/s).
  const bool tail_bound = offs[n] - offs[0] > (uint64_t)n * kWaveCap;
  std::vector<size_t> cut{0};
  while (cut.back() < n) {
    const size_t a = cut.back();
    const size_t ci = cut.size() - 1;
    const uint64_t kChunkBytes = tail_bound ? 4 * chunk_bytes()
                                            : std::max<uint64_t>(1u << 20, chunk_bytes() >> (ci < 3 ? 3 - ci : 0));
    const size_t kChunkDocs = (size_t)(kChunkBytes >> 7);    // 8K documents per MB
    size_t lo = a + 1, hi = std::min(n, a + kChunkDocs);     // largest b <= hi with bytes <= kChunkBytes (>= 1 doc)
    while (lo < hi) {
      const size_t mid = (lo + hi + 1) / 2;
      if (offs[mid] - offs[a] <= kChunkBytes) lo = mid; else hi = mid - 1;
    }
    cut.push_back(lo);
  }
  const size_t nch = cut.size() - 1;
  if (grow_host(&d->h_ctr, &d->h_ctr_cap, nch * kCtrSlots)) return CLD_ENOMEM;
  if (grow(&d->d_ctrs, &d->ctrs_cap, nch * kCtrSlots)) return CLD_ENOMEM;
  // every chunk's counters zeroed at once here, read back at once after the loop
  HIP_OK(hipMemsetAsync(d->d_ctrs, 0, nch * kCtrSlots * sizeof(uint32_t), d->stream));
  // both slots sized for the largest chunk up front (the previous call has
  // drained, so no buffer is reallocated under a running copy or kernel)
  size_t max_m = 0;
  uint64_t max_bytes = 1;
  for (size_t c = 0; c < nch; ++c) {
    max_m = std::max(max_m, cut[c + 1] - cut[c]);
    max_bytes = std::max<uint64_t>(max_bytes, offs[cut[c + 1]] - offs[cut[c]]);
  }
  for (Device::Slot& h : d->hs) {
    int r = grow(&h.d_in, &h.d_in_cap, max_bytes);
    if (!r) r = grow(&h.d_offs, &h.d_offs_cap, max_m + 1);
    if (!r) r = grow(&h.d_out, &h.d_out_cap, max_m);
    if (!r && !in_pinned) r = grow_host(&h.h_in, &h.h_in_cap, max_bytes);
    if (!r && !in_pinned) r = grow_host(&h.h_offs, &h.h_offs_cap, max_m + 1);
    if (!r && !out_pinned) r = grow_host(&h.h_out, &h.h_out_cap, max_m);
    if (!r && special) r = grow(&h.d_sp, &h.d_sp_cap, max_m);
    if (!r && special) r = grow_host(&h.h_sp, &h.h_sp_cap, max_m);
    if (!r && priors) r = grow(&h.d_pri, &h.d_pri_cap, 16 * max_m);
    if (!r && priors) r = grow_host(&h.h_pri, &h.h_pri_cap, 16 * max_m);
    if (r) return r;
  }
  int rc = CLD_OK;
  auto deliver = [&](Device::Slot& h) -> int {
    if (!h.busy) return CLD_OK;
    HIP_OK(hipEventSynchronize(h.down));
    if (h.pending_dst && h.pending_dst != h.h_out) par_copy(h.pending_dst, h.h_out, h.pending_n * sizeof(cld_result));
    h.busy = false;
    return CLD_OK;
  };
  // Per chunk c in slot c&1: once chunk c-2's UPLOAD is done its pinned
  // staging is free, so chunk c is staged while the GPU still runs c-2 and
  // c-1; c-2's results are handed over just before c's download reuses h_out.
  for (size_t c = 0; c < nch && rc == CLD_OK; ++c) {
    Device::Slot& h = d->hs[c & 1];
    if (h.busy) HIP_BRK(hipEventSynchronize(h.up))
    const size_t a = cut[c], m = cut[c + 1] - a;
    const uint64_t base = offs[a], bytes = offs[a + m] - base;
    const uint8_t* src_in = buf + base;
    const uint64_t* src_offs = offs + a;
    if (!in_pinned) {
      par_copy(h.h_in, src_in, bytes);
      memcpy(h.h_offs, src_offs, (m + 1) * sizeof(uint64_t));
      src_in = h.h_in;
      src_offs = h.h_offs;
    }
    cld_result* dst = out + a;
    if (special) {           // per-document routing bits (and priors) for this chunk, staged pinned
      memcpy(h.h_sp, special + a, m);
      if (priors) memcpy(h.h_pri, priors + 16 * a, 16 * m * sizeof(uint32_t));
    }
    // upload (after the slot's previous kernels stopped reading its device buffers)
    HIP_BRK(hipStreamWaitEvent(d->up_stream, h.comp, 0))
    if (bytes) HIP_BRK(hipMemcpyAsync(h.d_in, src_in, bytes, hipMemcpyHostToDevice, d->up_stream))
    HIP_BRK(hipMemcpyAsync(h.d_offs, src_offs, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, d->up_stream))
    if (special) {
      HIP_BRK(hipMemcpyAsync(h.d_sp, h.h_sp, m, hipMemcpyHostToDevice, d->up_stream))
      if (priors)
        HIP_BRK(hipMemcpyAsync(h.d_pri, h.h_pri, 16 * m * sizeof(uint32_t), hipMemcpyHostToDevice, d->up_stream))
    }
    HIP_BRK(hipEventRecord(h.up, d->up_stream))
    // kernels: buffer base biased so that the caller's offsets index it directly.
    // They write h.d_out, which chunk c-2's download may still be reading on
    // down_stream: wait for that copy on the device (the host hand-over of its
    // results, deliver() below, comes later and keeps the overlap).
    HIP_BRK(hipStreamWaitEvent(d->stream, h.up, 0))
    if (h.busy) HIP_BRK(hipStreamWaitEvent(d->stream, h.down, 0))
    const uint8_t* kbuf = h.d_in - base;
    // documents of this chunk longer than k_wave takes (counted up to the
    // small-list bound; StripExtras only shortens documents); one over the
    // fused kernel's cap needs the staged path whatever the count
    int64_t long_hint = 0;
    {
      const int64_t lim = (int64_t)small_long_list(d);
      const uint64_t* o = offs + a;
      const uint64_t heavy = small_list_heavy_bytes();
      for (size_t i = 0; i < m && long_hint <= lim; ++i) {
        const uint64_t len = o[i + 1] - o[i];
        long_hint += len > (uint64_t)kWaveCap;
        if (len > kLongDocCap - 64 || len >= heavy) long_hint = lim + 1;
      }
    }
    if (flags & kPrepFlags) {
      if ((rc = enqueue_prepare(d, kbuf, h.d_offs, m, bytes, flags, d->stream))) break;
      rc = enqueue(d, d->d_sbuf, d->d_soffs, m, h.d_out, d->stream, nullptr, nullptr, flags, 0, 0,
                   d->d_ctrs + c * kCtrSlots, long_hint);
    } else {
      rc = enqueue(d, kbuf, h.d_offs, m, h.d_out, d->stream, special ? h.d_sp : nullptr,
                   (special && priors) ? h.d_pri : nullptr, flags, base, (special && html) ? bytes : 0,
                   d->d_ctrs + c * kCtrSlots, long_hint);
    }
    if (rc) break;
    HIP_BRK(hipEventRecord(h.comp, d->stream))
    // download (chunk c-2's results out of h_out first)
    if ((rc = deliver(h))) break;
    HIP_BRK(hipStreamWaitEvent(d->down_stream, h.comp, 0))
    HIP_BRK(hipMemcpyAsync(out_pinned ? dst : h.h_out, h.d_out, m * sizeof(cld_result), hipMemcpyDeviceToHost,
                          d->down_stream))
    HIP_BRK(hipEventRecord(h.down, d->down_stream))
    h.pending_n = m;
    h.pending_dst = out_pinned ? nullptr : dst;
    h.busy = true;
  }
  if (rc == CLD_OK && d->h_trace) watch_trace(d, d->stream);
  if (rc == CLD_OK && hipMemcpyAsync(d->h_ctr, d->d_ctrs, nch * kCtrSlots * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                     d->stream) != hipSuccess)
    rc = CLD_EFAULT;
  for (auto& h : d->hs) {                              // drain (also after an error: no DMA may outlive the call)
    int r = deliver(h);
    if (rc == CLD_OK) rc = r;
  }
  // an upload or a kernel enqueued before an error in the loop may still read
  // the caller's (possibly registered) buffers: all three streams drain
  // before the HostReg objects above unregister them
  for (hipStream_t q : {d->up_stream, d->stream, d->down_stream})
    if (hipStreamSynchronize(q) != hipSuccess && rc == CLD_OK) rc = CLD_EFAULT;
  if (rc) return rc;
  if (d->d_dbg) {             // debug: write the dumped words to $CLD_DEBUG_OUT
    uint32_t cnt = 0;
    HIP_OK(hipMemcpy(&cnt, d->d_dbg, 4, hipMemcpyDeviceToHost));
    cnt = std::min<uint32_t>(cnt, (64u << 18) - 1);
    std::vector<uint32_t> w(cnt + 1);
    HIP_OK(hipMemcpy(w.data(), d->d_dbg, 4ull * (cnt + 1), hipMemcpyDeviceToHost));
    const char* path = getenv("CLD_DEBUG_OUT") ? getenv("CLD_DEBUG_OUT") : "/tmp/cld_dbg.bin";
    if (FILE* f = fopen(path, "wb")) { fwrite(w.data(), 4, w.size(), f); fclose(f); }
  }
  // statistics of the whole call: counters summed over chunks, kernel time over launches
  cld_batch_stats& st = d->last;
  memset(&st, 0, sizeof(st));
  bool err = false;
  for (size_t c = 0; c < nch; ++c) {
    add_counters(d, d->h_ctr + c * kCtrSlots, cut[c + 1] - cut[c], &st);
    err |= d->h_ctr[c * kCtrSlots + kCtrError] != 0;
  }
  for (size_t i = 0; i < d->ev_used; ++i) {
    float x = 0, y = 0, z = 0;
    HIP_OK(hipEventElapsedTime(&x, d->ev_pool[i][0], d->ev_pool[i][1]));
    HIP_OK(hipEventElapsedTime(&y, d->ev_pool[i][1], d->ev_pool[i][2]));
    HIP_OK(hipEventElapsedTime(&z, d->ev_pool[i][2], d->ev_pool[i][3]));
    st.short_ms += x; st.long_ms += y; st.general_ms += z;
  }
  d->stats_pending = false;
  return err ? kDocsFailed : CLD_OK;
}

// Request-sized batches of short documents: the per-call cost the reference's
// per-document wrapper call (wrapper.cc:7-16, handlers.go:132-151) would
// otherwise pay in full -- the streamed path's six launches, three streams,
// chunk events and counter copies -- is cut to one upload, one k_wave launch,
// one download and one synchronisation, on a tiny slot of its own (its own
// stream, pinned block and re-queue list; none of the context's scratch, so
// it needs neither the context lock nor the `done` chain).  Documents k_wave
// re-queues (a second script span, a second hit round, ...) are redone on the
// streamed path; results are the same whichever path finishes a document.
// CLD_TINY=0 turns it off (A/B).
bool tiny_enabled() {
  static const bool v = !(getenv("CLD_TINY") && atoi(getenv("CLD_TINY")) == 0);
  return v;
}

bool tiny_batch(const Device* d, const uint64_t* offs, size_t n, uint32_t flags, const uint8_t* special,
                const uint32_t* priors) {
  if (n == 0 || n > kTinyDocs || special || priors || (flags & kPrepFlags) || !tiny_enabled()) return false;
  if (d->d_dbg || d->h_trace || d->d_prof || d->fault_doc != 0xFFFFFFFFu) return false;   // diagnostics
  uint64_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad |= (uint64_t)(offs[i + 1] - offs[i] > (uint64_t)kWaveCap);
  return bad == 0;
}

// CLD_TINY_ZC=1: k_wave reads the documents from the pinned block and
// writes the results into it over PCIe (no DMA at all: one launch and one
// synchronisation per call); default: one upload and one download.
bool tiny_zero_copy() {
  static const bool v = getenv("CLD_TINY_ZC") && atoi(getenv("CLD_TINY_ZC")) != 0;
  return v;
}

struct DocRef {
  const uint8_t* p;
  size_t len;
};

// k_wave alone over n documents of at most kWaveCap bytes in tiny slot t (the
// caller holds t->mu): doc(i) -> DocRef, written straight into the slot's
// pinned block.  Results in out; the documents k_wave hands on come back
// marked kWaveRequeued (no counters).
template <class DocFn>
int tiny_run_slot(Device* d, TinySlot* t, size_t n, DocFn doc, cld_result* out, uint32_t flags) {
  HIP_OK(hipSetDevice(d->id));
  const size_t text_off = kTinyOffsOff + (n + 1) * sizeof(uint64_t);
  const size_t out_off = kTinyCtrOff - n * sizeof(cld_result);
  uint64_t* ho = (uint64_t*)(t->h + kTinyOffsOff);
  uint8_t* ht = t->h + text_off;
  uint64_t bytes = 0;
  for (size_t i = 0; i < n; ++i) {
    const DocRef r = doc(i);
    ho[i] = bytes;
    memcpy(ht + bytes, r.p, r.len);
    bytes += r.len;
  }
  ho[n] = bytes;
  if (tiny_zero_copy()) {
    HIP_OK(cld_launch_wave_only(&d->T, t->hd + text_off, (const uint64_t*)(t->hd + kTinyOffsOff), (int)n,
                                (cld_result*)(t->hd + out_off), nullptr, nullptr, flags & kCldFlags, t->s));
  } else {
    HIP_OK(hipMemcpyAsync(t->dv + kTinyOffsOff, t->h + kTinyOffsOff, text_off - kTinyOffsOff + bytes,
                          hipMemcpyHostToDevice, t->s));
    HIP_OK(cld_launch_wave_only(&d->T, t->dv + text_off, (const uint64_t*)(t->dv + kTinyOffsOff), (int)n,
                                (cld_result*)(t->dv + out_off), nullptr, nullptr, flags & kCldFlags, t->s));
    HIP_OK(hipMemcpyAsync(t->h + out_off, t->dv + out_off, n * sizeof(cld_result), hipMemcpyDeviceToHost, t->s));
  }
  HIP_OK(hipStreamSynchronize(t->s));
  memcpy(out, t->h + out_off, n * sizeof(cld_result));
  return CLD_OK;
}

// The documents of a tiny call that k_wave handed on (kWaveRequeued), gathered
// and redone on the streamed path; *st gets the call's statistics.
template <class DocFn>
int tiny_redo_requeued(Device* d, size_t n, DocFn doc, cld_result* out, uint32_t flags, cld_batch_stats* st) {
  std::vector<uint32_t> list;
  for (size_t i = 0; i < n; ++i)
    if (out[i].summary_lang == kWaveRequeued) list.push_back((uint32_t)i);
  const uint32_t rq = (uint32_t)list.size();
  *st = cld_batch_stats{};
  st->docs = n;
  st->short_docs = n - rq;
  st->passes[0] = n - rq;
  if (rq == 0) return CLD_OK;
  std::vector<uint8_t> gb;
  std::vector<uint64_t> go{0};
  for (uint32_t i : list) {
    const DocRef r = doc(i);
    gb.insert(gb.end(), r.p, r.p + r.len);
    go.push_back(gb.size());
  }
  std::vector<cld_result> gout(rq);
  const int rc = run_host_stream(d, gb.data(), go.data(), rq, gout.data(), flags);
  if (rc != CLD_OK && rc != kDocsFailed) return rc;
  for (uint32_t k = 0; k < rq; ++k) out[list[k]] = gout[k];
  std::lock_guard<std::mutex> dl(d->mu);
  const cld_batch_stats s2 = d->last;                  // the streamed call's counts for the re-queued documents
  st->long_docs = s2.long_docs;
  st->general_docs = s2.general_docs;
  st->short_docs += s2.short_docs;
  for (int k = 0; k < 4; ++k) st->passes[k] += s2.passes[k];
  for (int k = 0; k < 8; ++k) st->long_requeue[k] = s2.long_requeue[k];
  st->short_ms = s2.short_ms; st->long_ms = s2.long_ms; st->general_ms = s2.general_ms;
  return rc;
}

int run_tiny(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out, uint32_t flags) {
  TinySlot* t = nullptr;
  std::unique_lock<std::mutex> lk;
  const int ns = tiny_slots();
  for (int k = 0; k < ns; ++k) {
    std::unique_lock<std::mutex> l(d->tiny[k].mu, std::try_to_lock);
    if (l.owns_lock()) { t = &d->tiny[k]; lk = std::move(l); break; }
  }
  if (!t) {
    t = &d->tiny[d->tiny_rr.fetch_add(1) % ns];
    lk = std::unique_lock<std::mutex>(t->mu);
  }
  auto doc = [&](size_t i) { return DocRef{buf + offs[i], (size_t)(offs[i + 1] - offs[i])}; };
  if (int rc = tiny_run_slot(d, t, n, doc, out, flags)) return rc;
  lk.unlock();
  cld_batch_stats st{};
  const int rc = tiny_redo_requeued(d, n, doc, out, flags, &st);
  if (rc != CLD_OK && rc != kDocsFailed) return rc;
  if (st.docs == st.short_docs) {
    std::unique_lock<std::mutex> dl(d->mu, std::try_to_lock);   // best effort: diagnostics only
    if (dl.owns_lock()) { d->last = st; d->stats_pending = false; }
  } else {
    std::lock_guard<std::mutex> dl(d->mu);
    d->last = st;
  }
  return rc;
}

// One device's share of a host batch: run_tiny when it qualifies, else the streamed path.
int run_host_shard(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out, uint32_t flags,
                   const uint8_t* special = nullptr, const uint32_t* priors = nullptr, bool html = false) {
  if (tiny_batch(d, offs, n, flags, special, priors)) return run_tiny(d, buf, offs, n, out, flags);
  return run_host_stream(d, buf, offs, n, out, flags, special, priors, html);
}

// Documents the kernels could not score come back marked CLD_LANG_FAILED
// (k_long, kDocsFailed above); each is redone alone, so one bad document
// never costs the batch.  CLD_EIO only if one still fails on its own.
// The failed documents are retried together, as one gathered batch (scoring
// is deterministic: outside fault injection a document that failed fails
// again, so a batch with many marked documents must not turn into one GPU
// round trip per document).  Only when the gathered retry itself reports
// failures, and at most kIsolateAlone of them, is each such document run
// alone, so one document cannot take another's result with it.
constexpr size_t kIsolateAlone = 16;
int run_host_shard_isolating(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out,
                             uint32_t flags, const uint8_t* special = nullptr, const uint32_t* priors = nullptr,
                             bool html = false) {
  int rc = run_host_shard(d, buf, offs, n, out, flags, special, priors, html);
  if (rc != kDocsFailed) return rc;
  std::vector<size_t> idx;
  for (size_t i = 0; i < n; ++i)
    if (out[i].summary_lang == CLD_LANG_FAILED) idx.push_back(i);
  // gather the failed documents (with their routing bits and priors) into one batch
  std::vector<uint8_t> gb;
  std::vector<uint64_t> go{0};
  std::vector<uint8_t> gsp;
  std::vector<uint32_t> gpr;
  for (size_t i : idx) {
    gb.insert(gb.end(), buf + offs[i], buf + offs[i + 1]);
    go.push_back(gb.size());
    if (special) gsp.push_back(special[i]);
    if (priors) gpr.insert(gpr.end(), priors + 16 * i, priors + 16 * i + 16);
  }
  std::vector<cld_result> gout(idx.size());
  int r = run_host_shard(d, gb.data(), go.data(), idx.size(), gout.data(), flags, special ? gsp.data() : nullptr,
                         priors ? gpr.data() : nullptr, html);
  if (r != CLD_OK && r != kDocsFailed) return r;          // a device error, not a document
  size_t left = 0;
  for (size_t k = 0; k < idx.size(); ++k) {
    out[idx[k]] = gout[k];
    if (gout[k].summary_lang != CLD_LANG_FAILED) continue;
    if (++left > kIsolateAlone) continue;                 // stays marked: CLD_EIO below
    const size_t i = idx[k];
    r = run_host_shard(d, buf, offs + i, 1, out + i, flags, special ? special + i : nullptr,
                       priors ? priors + 16 * i : nullptr, html);
    if (r != CLD_OK && r != kDocsFailed) return r;
    if (r == CLD_OK) --left;
  }
  if (left) fprintf(stderr, "cld_mi355x: %zu document(s) without a result after a retry (summary CLD_LANG_FAILED)\n", left);
  return left ? CLD_EIO : CLD_OK;
}

// Multi-GPU fan-out: large pageable caller buffers are page-locked once by
// the dispatching thread, so the shards (whose offset and result ranges share
// boundary entries and pages) find them pinned instead of each registering an
// overlapping range.
struct FanoutReg {
  HostReg b, o, r;
  FanoutReg(size_t ndev, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out) {
    if (ndev < 2 || offs[n] - offs[0] < register_min_bytes()) return;
    if (!host_pinned(buf + offs[0]) && b.take(buf + offs[0], offs[n] - offs[0]) && !host_pinned(offs))
      o.take(offs, (n + 1) * sizeof(uint64_t));
    if (!host_pinned(out)) r.take(out, n * sizeof(cld_result));
  }
};

// ResultChunkVector mode on one device: documents in sub-batches (the
// kernel is the exact sequential pipeline; no overlap needed), each
// document building its vector in a pool region of len + len/4 + 8 chunks,
// then a gather into document order.  Appends the chunks of documents
// [0, n) to *chunks and their counts to *counts.
int run_vec_shard(Device* d, const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out,
                  const uint8_t* special, const uint32_t* priors, std::vector<cld_chunk>* chunks,
                  std::vector<int32_t>* counts, uint32_t cflags) {
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  Device::Vec& V = d->vec;
  // k_long<VEC> builds every vector (the parallel span builder, or for the
  // documents it cannot formulate the sequential span source), one VecSlot per
  // resident wave, allocated on the first vector call
  if (!V.vslots && hipMalloc(&V.vslots, (uint64_t)d->n_slots * cld_vec_slot_bytes()) != hipSuccess) {
    V.vslots = nullptr;
    return CLD_ENOMEM;
  }
  // Sub-batches as large as memory allows: a launch lasts at least as long as
  // its longest document (one wave runs it start to end), so every sub-batch
  // pays that tail once -- 32 MB sub-batches held C5 to 76K docs/s, one launch
  // for the 95 MB batch runs it at 208K.  256 MB of text takes ~5 GB of pool.
  const size_t kSub = 1024 * 1024;
  static const uint64_t kSubBytes0 = (getenv("CLD_VEC_SUB_MB") ? (uint64_t)atoi(getenv("CLD_VEC_SUB_MB")) : 256ull) << 20;
  uint64_t kSubBytes = kSubBytes0;   // halved while the device cannot hold a sub-batch's pool
  // test hook: CLD_VEC_POOL_SMALL=1 makes first-pass pool regions too small so
  // the retry below runs (tests/test_gpu_vector.py)
  static const bool small_pool = getenv("CLD_VEC_POOL_SMALL") && atoi(getenv("CLD_VEC_POOL_SMALL")) > 0;
  // One sub-batch: documents [o[0], o[m]) of b (o: offsets into b), document
  // i building its vector in a pool region of len + len/4 + 8 chunks (big: 8 len
  // + 256); results to res, vector sizes to nch (-1: the document overflowed
  // its pool region or an offset map), the vectors to ch in document order.
  std::vector<uint64_t> pool_off, pos;
  cld_batch_stats vst{};
  auto sub = [&](const uint8_t* b, const uint64_t* o, size_t m, cld_result* res, const uint8_t* sp,
                 const uint32_t* pr, bool big, std::vector<int32_t>& nch, std::vector<cld_chunk>& ch) -> int {
    const uint64_t base = o[0], bytes = o[m] - base;
    pool_off.assign(m + 1, 0);
    for (size_t i = 0; i < m; ++i) {
      const uint64_t len = o[i + 1] - o[i];
      pool_off[i + 1] = pool_off[i] + (big ? 8 * len + 256 : small_pool ? 1 : len + len / 4 + 8);
    }
    if (grow(&V.in, &V.in_cap, std::max<size_t>(bytes, 1)) || grow(&V.offs, &V.offs_cap, m + 1) ||
        grow(&V.out, &V.out_cap, m) || grow(&V.pool, &V.pool_cap, pool_off[m]) ||
        grow(&V.pool_off, &V.pool_off_cap, m + 1) || grow(&V.nch, &V.nch_cap, m) || grow(&V.pos, &V.pos_cap, m))
      return CLD_ENOMEM;
    if (sp && grow(&V.sp, &V.sp_cap, m)) return CLD_ENOMEM;
    if (pr && grow(&V.pri, &V.pri_cap, 16 * m)) return CLD_ENOMEM;
    hipStream_t s = d->stream;
    HIP_OK(hipStreamWaitEvent(s, d->done, 0));
    if (bytes) HIP_OK(hipMemcpyAsync(V.in, b + base, bytes, hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(V.offs, o, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(V.pool_off, pool_off.data(), (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    if (sp) HIP_OK(hipMemcpyAsync(V.sp, sp, m, hipMemcpyHostToDevice, s));
    if (pr) HIP_OK(hipMemcpyAsync(V.pri, pr, 16 * m * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemsetAsync(d->d_counters, 0, kCtrSlots * sizeof(uint32_t), s));
    {
      if (grow(&d->d_requeue, &d->requeue_cap, m) || grow(&d->d_requeue2, &d->requeue2_cap, m) ||
          grow(&d->d_lsorted, &d->lsorted_cap, m) || grow(&d->d_lkey, &d->lkey_cap, m))
        return CLD_ENOMEM;
      // HTML pages: rewritten into plain text with each byte's page offset
      // (cld_html.hip), then scored by k_long<VEC> like plain documents
      const uint8_t* hb = nullptr;
      const uint8_t* hf = nullptr;
      const uint32_t* hpz = nullptr;
      const uint32_t* hgz = nullptr;
      if (sp) {
        if (grow(&d->d_hbuf, &d->hbuf_cap, std::max<size_t>(bytes, 1)) ||
            grow(&d->d_hflag, &d->hflag_cap, std::max<size_t>(bytes, 1)) ||
            grow(&d->d_hpos, &d->hpos_cap, 2 * std::max<size_t>(bytes, 1)))
          return CLD_ENOMEM;
        hb = d->d_hbuf - base;
        hf = d->d_hflag - base;
        hpz = d->d_hpos - base;
        hgz = d->d_hpos + std::max<size_t>(bytes, 1) - base;
        HIP_OK(cld_launch_html_rewrite(d->d_T, V.in - base, V.offs, (int)m, V.sp, const_cast<uint8_t*>(hb),
                                       const_cast<uint8_t*>(hf), const_cast<uint32_t*>(hpz),
                                       const_cast<uint32_t*>(hgz), 0, nullptr, s));
      }
      HIP_OK(cld_launch_route_vec((int)m, d->d_counters, d->d_requeue, s));
      HIP_OK(cld_launch_order_long(V.offs, d->d_requeue, d->d_counters, d->d_lkey, d->d_lhist, d->d_lsorted, false, s));
      HIP_OK(cld_launch_long_vec(d->d_T, V.in - base, V.offs, d->d_lsorted, V.out, d->d_slots, V.vslots, d->n_slots,
                                 d->d_requeue2, d->d_counters, cflags & kCldFlags, sp ? V.sp : nullptr, pr ? V.pri : nullptr, hb, hf,
                                 hpz, hgz, V.pool, V.pool_off, V.nch, s));
    }
    nch.resize(m);
    uint32_t ctr[kCtrSlots];
    HIP_OK(hipMemcpyAsync(ctr, d->d_counters, sizeof(ctr), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(res, V.out, m * sizeof(cld_result), hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(nch.data(), V.nch, m * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    // statistics (cld_last_batch_stats): documents the parallel span builder
    // finished (long_docs) and those the sequential span source took (general_docs)
    vst.docs += m;
    vst.general_docs += ctr[kCtrSeq];
    vst.long_docs += m - ctr[kCtrSeq];
    for (int k = 0; k < 3; ++k) vst.passes[k] += ctr[kCtrPass1 + k];
    vst.passes[3] += ctr[kCtrError];
    pos.assign(m, 0);
    uint64_t total = 0;
    for (size_t i = 0; i < m; ++i) {
      pos[i] = total;
      if (nch[i] > 0) total += (uint64_t)nch[i];
    }
    if (grow(&V.compact, &V.compact_cap, std::max<uint64_t>(total, 1))) return CLD_ENOMEM;
    HIP_OK(hipMemcpyAsync(V.pos, pos.data(), m * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIP_OK(cld_launch_vec_gather(V.pool, V.pool_off, V.nch, V.pos, (int)m, V.compact, s));   // (-1: no chunks)
    ch.resize(total);
    if (total) HIP_OK(hipMemcpyAsync(ch.data(), V.compact, total * sizeof(cld_chunk), hipMemcpyDeviceToHost, s));
    HIP_OK(hipEventRecord(d->done, s));
    HIP_OK(hipStreamSynchronize(s));
    return CLD_OK;
  };
  size_t a = 0;
  bool failed = false;
  while (a < n) {
    size_t m = 1;                                       // at least one document, then up to the limits
    while (a + m < n && m < kSub && offs[a + m + 1] - offs[a] <= kSubBytes) ++m;
    std::vector<int32_t> nch;
    std::vector<cld_chunk> ch;
    if (int rc = sub(buf, offs + a, m, out + a, special ? special + a : nullptr, priors ? priors + 16 * a : nullptr,
                     false, nch, ch)) {
      if (rc == CLD_ENOMEM && m > 1 && kSubBytes > (1u << 20)) {   // smaller sub-batches, same documents
        kSubBytes /= 2;
        continue;
      }
      return rc;
    }
    // A document whose vector did not fit runs again, alone with the others
    // that did not, with 8x the pool region; the rest of the batch is kept.
    std::vector<size_t> bad;
    for (size_t i = 0; i < m; ++i)
      if (nch[i] < 0) bad.push_back(i);
    if (!bad.empty()) {
      std::vector<uint8_t> rb, rsp;
      std::vector<uint64_t> ro{0};
      std::vector<uint32_t> rpr;
      for (size_t i : bad) {
        rb.insert(rb.end(), buf + offs[a + i], buf + offs[a + i + 1]);
        ro.push_back(rb.size());
        if (special) rsp.push_back(special[a + i]);
        if (priors) rpr.insert(rpr.end(), priors + 16 * (a + i), priors + 16 * (a + i + 1));
      }
      std::vector<cld_result> rres(bad.size());
      std::vector<int32_t> nch2;
      std::vector<cld_chunk> ch2;
      if (int rc = sub(rb.empty() ? buf : rb.data(), ro.data(), bad.size(), rres.data(),
                       special ? rsp.data() : nullptr, priors ? rpr.data() : nullptr, true, nch2, ch2))
        return rc;
      std::vector<cld_chunk> merged;
      merged.reserve(ch.size() + ch2.size());
      size_t c1 = 0, c2 = 0, j = 0;
      for (size_t i = 0; i < m; ++i) {
        if (j < bad.size() && bad[j] == i) {
          out[a + i] = rres[j];
          const int32_t k = nch2[j];
          if (k < 0) failed = true;                   // no vector: an empty one, and CLD_EIO
          const size_t kk = k > 0 ? (size_t)k : 0;
          merged.insert(merged.end(), ch2.begin() + c2, ch2.begin() + c2 + kk);
          c2 += kk;
          nch[i] = (int32_t)kk;
          ++j;
        } else {
          merged.insert(merged.end(), ch.begin() + c1, ch.begin() + c1 + nch[i]);
          c1 += (size_t)nch[i];
        }
      }
      ch.swap(merged);
    }
    chunks->insert(chunks->end(), ch.begin(), ch.end());
    counts->insert(counts->end(), nch.begin(), nch.end());
    a += m;
  }
  d->last = vst;
  d->stats_pending = false;
  return failed ? CLD_EIO : CLD_OK;
}

// ------------------------------------------------ detect_language batching
// Host copy of the tables: the CLDT at `tables_path` (or the default), unless
// a cld2 dynamic data file was loaded first (cld_load_data_*).  Caller holds g_init_mu.
int host_tables(const char* tables_path) {
  if (!g_tab.blob.empty()) return CLD_OK;
  g_base_path = tables_path ? tables_path : default_tables_path();
  int rc = load_tables(g_base_path.c_str(), &g_tab);
  if (rc) g_tab = HostTables();
  return rc;
}

// Replace the scoring tables by a cld2 dynamic data image (compact_lang_det_impl.cc:108-136:
// loadDataFromFile / loadDataFromRawAddress).  Unlike the reference, a failed
// load keeps the tables in use and returns an error instead of leaving none.
int load_dynamic(const uint8_t* data, size_t len, const std::string& label) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  std::unique_lock<std::shared_mutex> tl(g_swap_mu);   // no batch call is between its hints and its kernels
  int rc = host_tables(nullptr);
  if (rc) return rc;
  HostTables nt;
  std::string err;
  if (cld::cld2_data_to_cldt(data, len, g_tab.blob.data(), g_tab.blob.size(), &nt.blob, &err) != 0) {
    fprintf(stderr, "WARNING: Dynamic data loading failed. (%s)\n", err.c_str());
    return CLD_EINVAL;
  }
  if ((rc = parse_tables(&nt, label)) != CLD_OK) {
    fprintf(stderr, "WARNING: Dynamic data loading failed. (tables rejected)\n");
    return rc;
  }
  if ((rc = swap_tables_all(nt)) != CLD_OK) return rc;
  g_tab = std::move(nt);
  g_dynamic = true;
  return CLD_OK;
}

int swap_tables_all(const HostTables& nt) {
  std::vector<StagedTables> st(g_devs.size());
  for (size_t i = 0; i < g_devs.size(); ++i) {
    std::lock_guard<std::mutex> dl(g_devs[i]->mu);
    if (int rc = stage_tables(g_devs[i], nt, &st[i])) {
      for (size_t j = 0; j <= i; ++j) discard_tables(g_devs[j], &st[j]);
      fprintf(stderr, "cld_mi355x: table upload failed on device %d; the tables in use are kept\n", g_devs[i]->id);
      return rc;
    }
  }
  for (size_t i = 0; i < g_devs.size(); ++i) {       // cannot fail short of a device error
    std::lock_guard<std::mutex> dl(g_devs[i]->mu);
    if (int rc = commit_tables(g_devs[i], &st[i])) return rc;
  }
  return CLD_OK;
}


}  // namespace

extern "C" {

int cld_init(const char* tables_path, int n_devices) {
  if (g_ready.load(std::memory_order_acquire)) return CLD_OK;
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_inited) return g_init_rc;
  g_inited = true;
  int rc = host_tables(tables_path);
  if (rc) return g_init_rc = rc;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    fprintf(stderr, "cld_mi355x: no HIP device available\n");
    return g_init_rc = CLD_ENODEV;
  }
  if (n_devices <= 0 || n_devices > count) n_devices = count;
  if (const char* e = getenv("CLD_MI355X_DEVICES")) n_devices = std::max(1, std::min(count, atoi(e)));
  std::vector<int> ids;
  for (int i = 0; i < n_devices; ++i) ids.push_back(i);
  // CLD_MI355X_DEVICE_MAP="0,0": one context per listed HIP ordinal, repeats
  // allowed -- the multi-device fan-out of the batch entry points (one host
  // thread per context, each with its own streams, tables and scratch) then
  // runs on a one-GPU box too (tests/test_gpu_streams.py)
  if (const char* e = getenv("CLD_MI355X_DEVICE_MAP")) {
    ids.clear();
    for (const char* p = e; *p;) {
      char* end = nullptr;
      const long v = strtol(p, &end, 10);
      if (end == p || v < 0 || v >= count) return g_init_rc = CLD_EINVAL;
      ids.push_back((int)v);
      p = *end == ',' ? end + 1 : end;
      if (*end && *end != ',') return g_init_rc = CLD_EINVAL;
    }
    if (ids.empty()) return g_init_rc = CLD_EINVAL;
  }
  // CLD_MI355X_CONTEXTS=k: k contexts per GPU (own streams, scratch and k_long
  // slots), so concurrent request-sized calls run side by side on one GPU
  // instead of queueing behind each other's longest document (pick_context)
  int per = 1;
  if (const char* e = getenv("CLD_MI355X_CONTEXTS")) per = std::max(1, std::min(64, atoi(e)));
  for (int id : ids)
    for (int k = 0; k < per; ++k) {
      Device* d = new Device();
      d->id = id;
      if ((rc = init_device(d)) != CLD_OK) return g_init_rc = rc;
      g_devs.push_back(d);
    }
  g_ready.store(true, std::memory_order_release);
  return g_init_rc = CLD_OK;
}

int cld_init_device(const char* tables_path, int device) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_inited) return g_init_rc;
  g_inited = true;
  int rc = host_tables(tables_path);
  if (rc) return g_init_rc = rc;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return g_init_rc = CLD_ENODEV;
  Device* d = new Device();
  d->id = device;
  if ((rc = init_device(d)) != CLD_OK) return g_init_rc = rc;
  g_devs.push_back(d);
  g_ready.store(true, std::memory_order_release);
  return g_init_rc = CLD_OK;
}

int cld_stage_cycles(int ctx, uint64_t* cycles16) {
  if (!cycles16 || ctx < 0 || ctx >= (int)g_devs.size()) return CLD_EINVAL;
  Device* d = g_devs[ctx];
  if (!d->d_prof) { memset(cycles16, 0, 16 * sizeof(uint64_t)); return CLD_OK; }
  (void)hipSetDevice(d->id);
  HIP_OK(hipStreamSynchronize(d->stream));
  HIP_OK(hipMemcpy(cycles16, d->d_prof, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  HIP_OK(hipMemset(d->d_prof, 0, 16 * sizeof(unsigned long long)));
  return CLD_OK;
}

int cld_kernel_times(int ctx, double* ms3, int* launches) {
  if (ctx < 0 || ctx >= (int)g_devs.size() || !ms3) return CLD_EINVAL;
  Device* d = g_devs[ctx];
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  double a = 0, b = 0, c = 0;
  for (size_t i = 0; i < d->ev_used; ++i) {
    HIP_OK(hipEventSynchronize(d->ev_pool[i][3]));
    float x = 0, y = 0, z = 0;
    HIP_OK(hipEventElapsedTime(&x, d->ev_pool[i][0], d->ev_pool[i][1]));
    HIP_OK(hipEventElapsedTime(&y, d->ev_pool[i][1], d->ev_pool[i][2]));
    HIP_OK(hipEventElapsedTime(&z, d->ev_pool[i][2], d->ev_pool[i][3]));
    a += x; b += y; c += z;
  }
  ms3[0] = a; ms3[1] = b; ms3[2] = c;
  if (launches) *launches = (int)d->ev_used;
  d->ev_used = 0;
  return CLD_OK;
}

int cld_kernel_time(int ctx, double* short_ms, double* general_ms, int* launches) {
  double ms[3];
  int rc = cld_kernel_times(ctx, ms, launches);
  if (rc) return rc;
  if (short_ms) *short_ms = ms[0];
  if (general_ms) *general_ms = ms[1] + ms[2];
  return CLD_OK;
}

// Estimated kernel cost of one document, in units of 10 ps, from this tree's
// measured per-document times on one MI355X:
//   <= 256 B   k_wave, one wavefront per document: 4.8 ms per 1 M tweets
//   longer     k_long: 84.4 ms per 100 K 16 KB pages = 0.0515 ns/B, plus
//              ~25 ns per document (C5's long half: 51.3 ms)
// so a 16 KB page weighs as much as ~180 tweets, not the ~110 that bytes +
// 64 per document said.
static uint64_t doc_cost(uint64_t len) { return len <= (uint64_t)kWaveCap ? 480 : (len * 41) / 8 + 2500; }

int cld_plan_shards(const uint64_t* offsets, size_t n, int nshards, size_t* cuts) {
  if (!offsets || !cuts || nshards < 1) return CLD_EINVAL;
  // Contiguous ranges of equal estimated kernel cost (doc_cost above): the
  // long-document kernel costs more per byte than the wavefront kernel, so a
  // byte split would leave the shard with the long pages last to finish.
  uint64_t total = 0;
  for (size_t i = 0; i < n; ++i) total += doc_cost(offsets[i + 1] - offsets[i]);
  cuts[0] = 0;
  uint64_t acc = 0;
  size_t i = 0;
  for (int k = 1; k < nshards; ++k) {
    const uint64_t target = (uint64_t)((unsigned __int128)total * (uint64_t)k / (uint64_t)nshards);
    while (i < n && acc < target) acc += doc_cost(offsets[i + 1] - offsets[i]), ++i;
    cuts[k] = i;
  }
  cuts[nshards] = n;
  return CLD_OK;
}

namespace {
void dl_stop();
}
void cld_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  std::unique_lock<std::shared_mutex> tl(g_swap_mu);
  dl_stop();
  for (Device* d : g_devs) {
    (void)hipSetDevice(d->id);
    (void)hipStreamSynchronize(d->stream);
    (void)hipFree(d->d_blob); (void)hipFree((void*)d->T.cpt); (void)hipFree((void*)d->T.keytab); (void)hipFree((void*)d->T.compat.adds); (void)hipFree(d->d_T); (void)hipFree(d->d_arena); (void)hipFree(d->d_counters);
    (void)hipFree(d->d_requeue); (void)hipFree(d->d_requeue2); (void)hipFree(d->d_lsorted); (void)hipFree(d->d_lkey); (void)hipFree(d->d_lhist); (void)hipFree(d->d_slots); (void)hipFree(d->d_buf); (void)hipFree(d->d_offs); (void)hipFree(d->d_out);
    (void)hipFree(d->d_sbuf); (void)hipFree(d->d_soffs); (void)hipFree(d->d_sscr);
    (void)hipFree(d->d_hbuf); (void)hipFree(d->d_hflag); (void)hipFree(d->d_hpos);
    (void)hipFree(d->d_spec_out); (void)hipFree(d->d_spec_take);
    (void)hipFree(d->d_store); (void)hipFree(d->d_meta); (void)hipFree(d->d_stlists); (void)hipFree(d->d_parlists);
    for (auto& t : d->ev_pool) for (auto& e : t) (void)hipEventDestroy(e);
    for (auto& h : d->hs) {
      (void)hipHostFree(h.h_in); (void)hipHostFree(h.h_offs); (void)hipHostFree(h.h_out);
      (void)hipFree(h.d_in); (void)hipFree(h.d_offs); (void)hipFree(h.d_out);
      (void)hipHostFree(h.h_sp); (void)hipHostFree(h.h_pri); (void)hipFree(h.d_sp); (void)hipFree(h.d_pri);
      (void)hipEventDestroy(h.up); (void)hipEventDestroy(h.comp); (void)hipEventDestroy(h.down);
    }
    (void)hipHostFree(d->h_ctr);
    (void)hipFree(d->d_ctrs);
    for (void* p : {(void*)d->vec.arena, (void*)d->vec.vslots, (void*)d->vec.in, (void*)d->vec.offs, (void*)d->vec.out, (void*)d->vec.sp,
                    (void*)d->vec.pri, (void*)d->vec.pool, (void*)d->vec.pool_off, (void*)d->vec.nch,
                    (void*)d->vec.pos, (void*)d->vec.order, (void*)d->vec.compact})
      if (p) (void)hipFree(p);
    for (TinySlot& t : d->tiny) {
      if (t.s) (void)hipStreamSynchronize(t.s);
      (void)hipHostFree(t.h); (void)hipFree(t.dv); (void)hipFree(t.d_rq);
      if (t.s) (void)hipStreamDestroy(t.s);
    }
    (void)hipEventDestroy(d->done);
    (void)hipStreamDestroy(d->up_stream);
    (void)hipStreamDestroy(d->down_stream);
    (void)hipStreamDestroy(d->stream);
    delete d;
  }
  g_devs.clear();
  g_tab = HostTables();
  g_dynamic = false;
  g_inited = false;
  g_ready.store(false, std::memory_order_release);
  g_init_rc = CLD_ENODEV;
}

namespace {
// A device error of any shard wins over CLD_EIO (some documents without a
// result, every other one complete).
int first_error(const std::vector<int>& rcs) {
  int partial = CLD_OK;
  for (int r : rcs) {
    if (r == CLD_EIO) partial = CLD_EIO;
    else if (r) return r;
  }
  return partial;
}
}  // namespace

namespace {
// Batches below this much text (CLD_SMALL_BATCH_MB, default 16) run whole on
// one context -- the least busy one -- instead of being split across all of
// them: a request-sized batch gains nothing from a split (its time is its
// longest document's), and concurrent callers then each get a context.
uint64_t small_batch_bytes() {
  static const uint64_t v = (getenv("CLD_SMALL_BATCH_MB") ? strtoull(getenv("CLD_SMALL_BATCH_MB"), nullptr, 10) : 16ull)
                            << 20;
  return v;
}
struct Picked {
  Device* d;
  explicit Picked(Device* x) : d(x) { d->inflight.fetch_add(1); }
  ~Picked() { d->inflight.fetch_sub(1); }
};
Device* pick_context();

// Request coalescing (cld_detect_batch below small_batch_bytes()).  A launch
// lasts as long as its longest document (one wavefront scores it start to
// end), so request-sized calls queued one after another cost that tail each;
// run together they pay it once.  The first caller to find a dispatch slot
// free (one per context) takes the queued requests with its flags, up to
// kCoalesceBytes of text / kCoalesceDocs documents, copies them into pinned
// buffers (the GPU reads those directly), runs them as one batch on the least
// busy context and hands every caller its results and return code.  A lone
// request runs straight from the caller's buffers.  Results never depend on
// the company a document keeps.
constexpr uint64_t kCoalesceBytes = 64ull << 20;
constexpr size_t kCoalesceDocs = 256 * 1024;
using cld::CoReq;
bool tiny_request(const uint64_t* offs, size_t n, uint32_t flags) {
  if (n > kTinyDocs || (flags & kPrepFlags) || !tiny_enabled()) return false;
  uint64_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad |= (uint64_t)(offs[i + 1] - offs[i] > (uint64_t)kWaveCap);
  return bad == 0;
}
struct Arena {                  // pinned staging of one dispatch (reused)
  uint8_t* buf = nullptr; size_t buf_cap = 0;
  uint64_t* offs = nullptr; size_t offs_cap = 0;
  cld_result* out = nullptr; size_t out_cap = 0;
};
std::mutex g_arena_mu;
std::vector<Arena*> g_arenas;   // free arenas

void run_group(const std::vector<CoReq*>& grp, void*) {
  if (grp.size() == 1) {        // nothing to merge: straight from the caller's buffers
    CoReq* r = grp[0];
    Picked p(pick_context());
    r->rc = run_host_shard_isolating(p.d, r->buf, r->offs, r->n, (cld_result*)r->out, r->flags);
    return;
  }
  Arena* a = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_arena_mu);
    if (!g_arenas.empty()) { a = g_arenas.back(); g_arenas.pop_back(); }
  }
  if (!a) a = new Arena();
  size_t docs = 0;
  uint64_t bytes = 0;
  for (CoReq* r : grp) { docs += r->n; bytes += r->offs[r->n] - r->offs[0]; }
  int rc = CLD_OK;
  if (grow_host(&a->buf, &a->buf_cap, std::max<uint64_t>(bytes, 1)) || grow_host(&a->offs, &a->offs_cap, docs + 1) ||
      grow_host(&a->out, &a->out_cap, docs))
    rc = CLD_ENOMEM;
  if (rc == CLD_OK) {
    size_t k = 0;
    uint64_t at = 0;
    for (CoReq* r : grp) {
      const uint64_t b0 = r->offs[0], nb = r->offs[r->n] - b0;
      memcpy(a->buf + at, r->buf + b0, nb);
      for (size_t i = 0; i < r->n; ++i) a->offs[k + i] = at + (r->offs[i] - b0);
      k += r->n;
      at += nb;
    }
    a->offs[docs] = at;
    Picked p(pick_context());
    rc = run_host_shard_isolating(p.d, a->buf, a->offs, docs, a->out, grp[0]->flags);
  }
  size_t k = 0;
  for (CoReq* r : grp) {
    cld_result* ro = (cld_result*)r->out;
    if (rc == CLD_OK || rc == CLD_EIO) {
      memcpy(ro, a->out + k, r->n * sizeof(cld_result));
      bool failed = false;
      for (size_t i = 0; i < r->n && rc == CLD_EIO; ++i) failed |= ro[i].summary_lang == CLD_LANG_FAILED;
      r->rc = failed ? CLD_EIO : CLD_OK;
    } else {
      r->rc = rc;
    }
    k += r->n;
  }
  std::lock_guard<std::mutex> lk(g_arena_mu);
  g_arenas.push_back(a);
}

// Dispatch slots (cld_coalesce.h): one per context for any group, and up to
// tiny_slots() per context while the extra ones carry tiny groups (run_tiny:
// each tiny slot has its own stream and buffers, so two such calls overlap on
// one GPU -- one uploads or synchronises while the other's kernel runs).
// Waiters sleep at once (CLD_COALESCE_SPIN_US: spin that long first): on a
// CPU-quota'd host (16 cores on the GPU box), spinning callers used up the
// quota and the cgroup throttled the whole process for the rest of its
// 100 ms period (gpurun_out/r5d).
cld::Coalescer* coalescer() {
  static cld::Coalescer* c = [] {
    cld::Coalescer* x = new cld::Coalescer();   // never destroyed (callers may be parked at exit)
    x->run = run_group;
    x->tiny_docs = kTinyDocs;
    x->max_bytes = kCoalesceBytes;
    x->max_docs = kCoalesceDocs;
    x->spin_us = getenv("CLD_COALESCE_SPIN_US") ? atoi(getenv("CLD_COALESCE_SPIN_US")) : 0;
    // the dispatcher wakes every member itself (CLD_COALESCE_WAKE=tree: members
    // wake each other): 256 callers 146K -> 263K docs/s, p99 74 -> 20 ms (r5d)
    x->tree_wake = getenv("CLD_COALESCE_WAKE") && !strcmp(getenv("CLD_COALESCE_WAKE"), "tree");
    return x;
  }();
  return c;
}

int run_coalesced(const uint8_t* buf, const uint64_t* offs, size_t n, cld_result* out, uint32_t flags) {
  cld::Coalescer& co = *coalescer();
  co.slots_any.store((int)g_devs.size(), std::memory_order_relaxed);   // (fixed while g_swap_mu is held)
  co.slots_tiny.store((int)g_devs.size() * tiny_slots(), std::memory_order_relaxed);
  CoReq me(buf, offs, n, out, flags, tiny_request(offs, n, flags));
  return co.submit(&me);
}

// detect_language's per-call path (cld_dlqueue.h): dispatcher threads, CLD_DL_DISPATCHERS
// per context (default 4, at most tiny_slots()), each on tiny slot k of its
// context, started on the first call (detached: they sleep on a futex when
// idle) and stopped by cld_shutdown.  CLD_DL_QUEUE=0: the calls take the
// coalescer (A/B).  C2 tweets, detect_language per call (profiles/
// round6_dl_rate_ab.jsonl): 256 callers 158 K docs/s on the coalescer (CPU
// quota exhausted: 117 us of CPU per call, 24 s throttled) -> 1.09 M with 2
// dispatchers, 1.30 M with 4 (17 us of CPU per call); 64 callers 406 K ->
// 486 K; a lone caller 25.0 K -> 22.6 K (the handoff to a dispatcher), 24.5 K
// once a call with no other in flight runs on its caller's thread (dl_direct).
cld::DlQueue g_dlq;
int dl_dispatchers() {
  static const int v = std::max(1, std::min(tiny_slots(), getenv("CLD_DL_DISPATCHERS") ? atoi(getenv("CLD_DL_DISPATCHERS")) : 4));
  return v;
}
bool dl_queue_on() {
  static const bool v = !(getenv("CLD_DL_QUEUE") && atoi(getenv("CLD_DL_QUEUE")) == 0);
  return v;
}
// how long callers (while fewer than 16 calls are in flight) and idle dispatchers spin before sleeping
int dl_caller_spin_us() {
  static const int v = getenv("CLD_DL_SPIN_US") ? atoi(getenv("CLD_DL_SPIN_US")) : 30;
  return v;
}
int dl_dispatcher_spin_us() {
  static const int v = getenv("CLD_DL_IDLE_SPIN_US") ? atoi(getenv("CLD_DL_IDLE_SPIN_US")) : 100;
  return v;
}

constexpr size_t kDlStop = ~(size_t)0;     // a request that stops the dispatcher taking it (dl_stop)

void dl_dispatch(Device* d, int k) {
  TinySlot* t = &d->tiny[k];
  std::vector<cld::DlReq*> v, stops;
  std::vector<cld_result> out(kTinyDocs);
  for (;;) {
    v.clear();
    stops.clear();
    for (cld::DlReq* r = g_dlq.take(dl_dispatcher_spin_us()); r; r = r->next) (r->len == kDlStop ? stops : v).push_back(r);
    for (size_t a = 0; a < v.size(); a += kTinyDocs) {
      const size_t n = std::min(kTinyDocs, v.size() - a);
      cld::DlReq* const* g = v.data() + a;
      auto doc = [&](size_t i) { return DocRef{g[i]->p, g[i]->len}; };
      int rc;
      {
        std::lock_guard<std::mutex> lk(t->mu);
        rc = tiny_run_slot(d, t, n, doc, out.data(), 0);
      }
      if (rc == CLD_OK) {
        cld_batch_stats st{};
        rc = tiny_redo_requeued(d, n, doc, out.data(), 0, &st);
      }
      for (size_t i = 0; i < n; ++i) {
        *static_cast<cld_result*>(g[i]->res) = out[i];
        // a document without a result is redone alone by its caller
        g[i]->rc = rc == kDocsFailed ? (out[i].summary_lang == CLD_LANG_FAILED ? kDocsFailed : CLD_OK) : rc;
        g_dlq.done_one();
      }
      cld::finish_batch(g, n);
    }
    if (!stops.empty()) {                      // (every request of the batch is finished)
      for (size_t i = 0; i < stops.size(); ++i) g_dlq.done_one();
      cld::finish_batch(stops.data(), stops.size());
      return;
    }
  }
}

// A call with no other in flight, on the caller's thread: the first tiny
// slot free (none: false, the caller queues it).  *rc as a dispatcher sets it.
bool dl_direct(const char* t, size_t len, cld_result* res, int* rc) {
  Device* d = g_devs[0];
  for (int k = 0; k < dl_dispatchers(); ++k) {
    std::unique_lock<std::mutex> lk(d->tiny[k].mu, std::try_to_lock);
    if (!lk.owns_lock()) continue;
    auto doc = [&](size_t) { return DocRef{(const uint8_t*)t, len}; };
    int r = tiny_run_slot(d, &d->tiny[k], 1, doc, res, 0);
    lk.unlock();
    if (r == CLD_OK) {
      cld_batch_stats st{};
      r = tiny_redo_requeued(d, 1, doc, res, 0, &st);
    }
    *rc = r == kDocsFailed ? (res->summary_lang == CLD_LANG_FAILED ? kDocsFailed : CLD_OK) : r;
    return true;
  }
  return false;
}

// 0: not started, 1: dispatchers running, 2: off (diagnostics on some context).
std::atomic<int> g_dl_state{0};
std::mutex g_dl_mu;
int g_dl_threads = 0;

// Eligible: a document k_wave takes (<= kWaveCap bytes), no diagnostics on
// any context (they need the streamed path's launches).  The caller holds
// g_swap_mu (shared) or g_init_mu: the contexts are fixed.
bool dl_queue_takes(size_t len) {
  if (len > (size_t)kWaveCap || !dl_queue_on() || !tiny_enabled()) return false;
  int st = g_dl_state.load(std::memory_order_acquire);
  if (st == 0) {
    std::lock_guard<std::mutex> lk(g_dl_mu);
    st = g_dl_state.load();
    if (st == 0) {
      bool ok = true;
      for (Device* d : g_devs)
        if (d->d_dbg || d->h_trace || d->d_prof || d->fault_doc != 0xFFFFFFFFu) ok = false;
      if (ok) {
        for (Device* d : g_devs)
          for (int k = 0; k < dl_dispatchers(); ++k) std::thread(dl_dispatch, d, k).detach();
        g_dl_threads = (int)g_devs.size() * dl_dispatchers();
      }
      st = ok ? 1 : 2;
      g_dl_state.store(st, std::memory_order_release);
    }
  }
  return st == 1;
}

// cld_shutdown (g_swap_mu held exclusively: no call is in flight): one stop
// request per dispatcher, each waited for, before the contexts go.
void dl_stop() {
  std::lock_guard<std::mutex> lk(g_dl_mu);
  if (g_dl_state.load() == 1)
    for (int k = 0; k < g_dl_threads; ++k) {
      cld_result dummy{};
      cld::DlReq r(nullptr, kDlStop, &dummy);
      g_dlq.enter();
      g_dlq.push(&r);
      r.wait(0);
    }
  g_dl_threads = 0;
  g_dl_state.store(0);
}

Device* pick_context() {
  static std::atomic<unsigned> rr{0};
  const size_t n = g_devs.size();
  const unsigned start = rr.fetch_add(1);
  Device* best = g_devs[start % n];
  int bl = best->inflight.load();
  for (size_t i = 1; i < n && bl > 0; ++i) {
    Device* d = g_devs[(start + i) % n];
    const int l = d->inflight.load();
    if (l < bl) { bl = l; best = d; }
  }
  return best;
}
}  // namespace

int cld_detect_batch(const uint8_t* buf, const uint64_t* offsets, size_t n, cld_result* out, uint32_t flags) {
  if ((flags & ~(kPrepFlags | kPublicFlags)) != 0 || (n > 0 && (!buf || !offsets || !out))) return CLD_EINVAL;
  if (n == 0) return CLD_OK;
  if (n > 0x7FFFFFFFu) return CLD_EINVAL;
  if (!offsets_nondecreasing(offsets, n)) return CLD_EINVAL;
  int rc = cld_init(nullptr, 0);
  if (rc) return rc;
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  const size_t ndev = g_devs.size();
  if (offsets[n] - offsets[0] < small_batch_bytes()) return run_coalesced(buf, offsets, n, out, flags);
  if (ndev == 1) return run_host_shard_isolating(g_devs[0], buf, offsets, n, out, flags);
  // Shard by estimated kernel cost at document boundaries (cld_plan_shards).
  std::vector<size_t> cut(ndev + 1, 0);
  cld_plan_shards(offsets, n, (int)ndev, cut.data());
  FanoutReg reg(ndev, buf, offsets, n, out);
  std::vector<int> rcs(ndev, CLD_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < ndev; ++k) {
    if (cut[k + 1] == cut[k]) continue;
    th.emplace_back([&, k] {
      rcs[k] = run_host_shard_isolating(g_devs[k], buf, offsets + cut[k], cut[k + 1] - cut[k], out + cut[k], flags);
    });
  }
  for (auto& t : th) t.join();
  return first_error(rcs);
}

int cld_hint_priors(const uint8_t* doc, size_t len, int is_plain_text, const cld_hints* hints, int16_t* priors14,
                    uint32_t* boosts16) {
  if ((!is_plain_text && len > 0 && !doc)) return CLD_EINVAL;
  {
    std::lock_guard<std::mutex> lk(g_init_mu);
    if (int rc = host_tables(nullptr)) return rc;
  }
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  const cld::HintView& v = g_tab.hints;
  if (!v.ok()) return CLD_EINVAL;               // tables without the hint sections
  int16_t p[cld::kMaxPriors] = {};
  const int n = cld::hint_priors(v, doc, len, is_plain_text != 0, hints, p);
  if (priors14) memcpy(priors14, p, sizeof(p));
  if (boosts16) cld::hint_boosts(v, p, n, boosts16);
  return n;
}

}  // extern "C"

namespace {
// ApplyHints per document on the host (a few table lookups, and for HTML a
// scan of the first 8 KB), split over host threads: the routing bits and,
// when any document has a prior, the 16 langprobs per document.  The caller
// holds g_swap_mu (shared).
int apply_hints(const uint8_t* buf, const uint64_t* offsets, size_t n, const cld_hints* hints, bool html,
                std::vector<uint8_t>* special, std::vector<uint32_t>* priors) {
  if (html && !g_tab.offs.ent_names) return CLD_EINVAL;     // tables without the HTML sections
  if ((html || hints) && !g_tab.hints.ok()) return CLD_EINVAL;
  special->assign(n, html ? kSpecialHtml : 0);
  priors->clear();
  if (!(html || hints)) return CLD_OK;
  priors->assign(16 * n, 0);
  std::atomic<bool> any(false);
  const int nt = (int)std::max<size_t>(1, std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()),
                                                           (n + 4095) / 4096));
  auto work = [&](size_t lo, size_t hi) {
    bool a = false;
    for (size_t i = lo; i < hi; ++i) {
      int16_t p[cld::kMaxPriors];
      const int k = cld::hint_priors(g_tab.hints, buf + offsets[i], offsets[i + 1] - offsets[i], !html,
                                     hints ? hints + i : nullptr, p);
      if (k <= 0) continue;
      uint32_t* o = priors->data() + 16 * i;
      cld::hint_boosts(g_tab.hints, p, k, o);
      bool nz = false;
      for (int j = 0; j < 16; ++j) nz |= o[j] != 0;
      if (nz) { (*special)[i] |= kSpecialPriors; a = true; }
    }
    if (a) any = true;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work, n * t / nt, n * (t + 1) / nt);
  work(0, n / nt);
  for (auto& x : th) x.join();
  if (!any) priors->clear();
  return CLD_OK;
}

int check_batch(const uint8_t* buf, const uint64_t* offsets, size_t n, const void* out) {
  if (n > 0 && (!buf || !offsets || !out)) return CLD_EINVAL;
  if (n > 0x7FFFFFFFu) return CLD_EINVAL;
  if (!offsets_nondecreasing(offsets, n)) return CLD_EINVAL;
  return CLD_OK;
}
}  // namespace

extern "C" {

int cld_detect_batch_ex(const uint8_t* buf, const uint64_t* offsets, size_t n, const cld_hints* hints,
                        uint32_t flags, cld_result* out) {
  if ((flags & ~(CLD_FLAG_HTML | kPublicFlags)) != 0) return CLD_EINVAL;
  if (int rc = check_batch(buf, offsets, n, out)) return rc;
  if (n == 0) return CLD_OK;
  int rc = cld_init(nullptr, 0);
  if (rc) return rc;
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  const uint32_t cf = flags & kCldFlags;
  std::vector<uint8_t> special;
  std::vector<uint32_t> priors;
  const bool html = (flags & CLD_FLAG_HTML) != 0;
  if ((rc = apply_hints(buf, offsets, n, hints, html, &special, &priors))) return rc;
  const uint8_t* sp = (html || !priors.empty()) ? special.data() : nullptr;
  const uint32_t* pr = priors.empty() ? nullptr : priors.data();
  const size_t ndev = g_devs.size();
  if (ndev == 1) return run_host_shard_isolating(g_devs[0], buf, offsets, n, out, cf, sp, pr, html);
  if (offsets[n] - offsets[0] < small_batch_bytes()) {
    Picked p(pick_context());
    return run_host_shard_isolating(p.d, buf, offsets, n, out, cf, sp, pr, html);
  }
  std::vector<size_t> cut(ndev + 1, 0);
  cld_plan_shards(offsets, n, (int)ndev, cut.data());
  FanoutReg reg(ndev, buf, offsets, n, out);
  std::vector<int> rcs(ndev, CLD_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < ndev; ++k) {
    if (cut[k + 1] == cut[k]) continue;
    th.emplace_back([&, k] {
      rcs[k] = run_host_shard_isolating(g_devs[k], buf, offsets + cut[k], cut[k + 1] - cut[k], out + cut[k], cf,
                              sp ? sp + cut[k] : nullptr, pr ? pr + 16 * cut[k] : nullptr, html);
    });
  }
  for (auto& t : th) t.join();
  return first_error(rcs);
}

int cld_detect_batch_vec(const uint8_t* buf, const uint64_t* offsets, size_t n, const cld_hints* hints,
                         uint32_t flags, cld_result* out, cld_chunk* chunks, size_t chunk_cap,
                         uint64_t* chunk_offsets) {
  if ((flags & ~(CLD_FLAG_HTML | kPublicFlags)) != 0 || !chunk_offsets || (chunk_cap > 0 && !chunks)) return CLD_EINVAL;
  if (int rc = check_batch(buf, offsets, n, out)) return rc;
  chunk_offsets[0] = 0;
  if (n == 0) return CLD_OK;
  int rc = cld_init(nullptr, 0);
  if (rc) return rc;
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  std::vector<uint8_t> special;
  std::vector<uint32_t> priors;
  const bool html = (flags & CLD_FLAG_HTML) != 0;
  if ((rc = apply_hints(buf, offsets, n, hints, html, &special, &priors))) return rc;
  const uint8_t* sp = (html || !priors.empty()) ? special.data() : nullptr;
  const uint32_t* pr = priors.empty() ? nullptr : priors.data();
  const size_t ndev = g_devs.size();
  std::vector<size_t> cut(ndev + 1, 0);
  cut[1] = n;
  if (ndev > 1) cld_plan_shards(offsets, n, (int)ndev, cut.data());
  std::vector<std::vector<cld_chunk>> vs(ndev);
  std::vector<std::vector<int32_t>> cs(ndev);
  std::vector<int> rcs(ndev, CLD_OK);
  std::vector<std::thread> th;
  for (size_t k = 0; k < ndev; ++k) {
    if (cut[k + 1] == cut[k]) continue;
    auto job = [&, k] {
      rcs[k] = run_vec_shard(g_devs[k], buf, offsets + cut[k], cut[k + 1] - cut[k], out + cut[k],
                             sp ? sp + cut[k] : nullptr, pr ? pr + 16 * cut[k] : nullptr, &vs[k], &cs[k],
                             flags & kCldFlags);
    };
    if (ndev == 1) job(); else th.emplace_back(job);
  }
  for (auto& t : th) t.join();
  int partial = CLD_OK;                 // CLD_EIO: some document got no vector; all others are complete
  for (int r : rcs) {
    if (r == CLD_EIO) partial = CLD_EIO;
    else if (r) return r;
  }
  size_t i = 0;
  uint64_t total = 0;
  for (size_t k = 0; k < ndev; ++k) {
    for (int32_t c : cs[k]) { total += (uint64_t)c; chunk_offsets[++i] = total; }
    const uint64_t at = total - vs[k].size();
    if (at < chunk_cap)
      memcpy(chunks + at, vs[k].data(), std::min<uint64_t>(vs[k].size(), chunk_cap - at) * sizeof(cld_chunk));
  }
  return total > chunk_cap ? CLD_ENOSPC : partial;
}

int cld_detect_batch_device(int device, const uint8_t* d_buf, const uint64_t* d_offsets, size_t n,
                            cld_result* d_out, void* stream) {
  int rc = cld_init(nullptr, 0);
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size()) return CLD_EINVAL;
  if (n == 0) return CLD_OK;
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  Device* d = g_devs[device];
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (d->ev_used >= 4096) d->ev_used = 0;     // bounded when callers never read timings
  return enqueue(d, d_buf, d_offsets, n, d_out, s);
}

int cld_detect_batch_device_ex(int device, const uint8_t* d_buf, const uint64_t* d_offsets, size_t n,
                               uint64_t buf_bytes, cld_result* d_out, uint32_t flags, void* stream) {
  if ((flags & ~(kPrepFlags | kPublicFlags)) != 0) return CLD_EINVAL;
  int rc = cld_init(nullptr, 0);
  if (rc) return rc;
  if (device < 0 || device >= (int)g_devs.size() || n > 0x7FFFFFFFu) return CLD_EINVAL;
  if (n == 0) return CLD_OK;
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  Device* d = g_devs[device];
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (d->ev_used >= 4096) d->ev_used = 0;
  if (!(flags & kPrepFlags)) return enqueue(d, d_buf, d_offsets, n, d_out, s, nullptr, nullptr, flags);
  if ((rc = enqueue_prepare(d, d_buf, d_offsets, n, buf_bytes, flags, s))) return rc;
  return enqueue(d, d->d_sbuf, d->d_soffs, n, d_out, s, nullptr, nullptr, flags);
}

int cld_prepare_batch(const uint8_t* buf, const uint64_t* offsets, size_t n, uint32_t flags,
                      uint8_t* out_buf, uint64_t* out_offsets) {
  if ((flags & ~kPrepFlags) != 0 || !offsets || !out_offsets || (n > 0 && (!buf || !out_buf))) return CLD_EINVAL;
  if (n > 0x7FFFFFFFu) return CLD_EINVAL;
  if (!offsets_nondecreasing(offsets, n)) return CLD_EINVAL;
  if (n == 0) { out_offsets[0] = 0; return CLD_OK; }
  int rc = cld_init(nullptr, 0);
  if (rc) return rc;
  Device* d = g_devs[0];
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  const uint64_t base = offsets[0], bytes = offsets[n] - offsets[0];
  if (grow(&d->d_buf, &d->buf_cap, std::max<size_t>(bytes, 1))) return CLD_ENOMEM;
  if (grow(&d->d_offs, &d->offs_cap, n + 1)) return CLD_ENOMEM;
  std::vector<uint64_t> rel(n + 1);
  for (size_t i = 0; i <= n; ++i) rel[i] = offsets[i] - base;
  if (bytes) HIP_OK(hipMemcpyAsync(d->d_buf, buf + base, bytes, hipMemcpyHostToDevice, d->stream));
  HIP_OK(hipMemcpyAsync(d->d_offs, rel.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, d->stream));
  if ((rc = enqueue_prepare(d, d->d_buf, d->d_offs, n, bytes, flags, d->stream))) return rc;
  HIP_OK(hipMemcpyAsync(out_offsets, d->d_soffs, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, d->stream));
  HIP_OK(hipStreamSynchronize(d->stream));
  if (out_offsets[n]) HIP_OK(hipMemcpy(out_buf, d->d_sbuf, out_offsets[n], hipMemcpyDeviceToHost));
  return CLD_OK;
}

int cld_last_batch_stats(int device, cld_batch_stats* st) {
  if (device < 0 || device >= (int)g_devs.size() || !st) return CLD_EINVAL;
  Device* d = g_devs[device];
  std::lock_guard<std::mutex> lk(d->mu);
  HIP_OK(hipSetDevice(d->id));
  int rc = collect_stats(d);
  *st = d->last;
  return rc;
}

void* cld_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void cld_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

const char* cld_language_code(int lang) {
  cld_init(nullptr, 0);
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  if (g_tab.codes.empty()) return "un";
  if (lang < 0 || (size_t)lang >= g_tab.codes.size()) lang = (int)g_tab.meta.unknown_language;
  return (size_t)lang < g_tab.codes.size() ? g_tab.codes[lang] : "un";
}

const char* cld_language_name(int lang) {
  cld_init(nullptr, 0);
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  if (g_tab.names.empty()) return "Unknown";
  if (lang < 0 || (size_t)lang >= g_tab.names.size()) lang = (int)g_tab.meta.unknown_language;
  return (size_t)lang < g_tab.names.size() ? g_tab.names[lang] : "Unknown";
}

const char* cld_version(void) {
  cld_init(nullptr, 0);
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  return intern(g_tab.version);
}

int cld_load_data_from_file(const char* path) {
  std::vector<uint8_t> data;
  if (!path || read_file(path, &data) != CLD_OK) {
    fprintf(stderr, "WARNING: Dynamic data loading failed. (cannot read %s)\n", path ? path : "(null)");
    return CLD_EINVAL;
  }
  return load_dynamic(data.data(), data.size(), std::string("cld2-data-file:") + path);
}

int cld_load_data_from_raw_address(const void* raw, uint32_t length) {
  if (!raw) return CLD_EINVAL;
  return load_dynamic((const uint8_t*)raw, length, "cld2-data-raw");
}

int cld_unload_data(void) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  std::unique_lock<std::shared_mutex> tl(g_swap_mu);
  if (!g_dynamic) return CLD_OK;
  HostTables nt;
  int rc = load_tables(g_base_path.c_str(), &nt);
  if (rc) return rc;
  if ((rc = swap_tables_all(nt)) != CLD_OK) return rc;
  g_tab = std::move(nt);
  g_dynamic = false;
  return CLD_OK;
}

int cld_is_data_dynamic(void) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  return g_dynamic ? 1 : 0;
}

int cld_export_tables(const char* out_path) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  int rc = host_tables(nullptr);
  if (rc) return rc;
  FILE* f = out_path ? fopen(out_path, "wb") : nullptr;
  if (!f) return CLD_EINVAL;
  size_t w = fwrite(g_tab.blob.data(), 1, g_tab.blob.size(), f);
  return (fclose(f) == 0 && w == g_tab.blob.size()) ? CLD_OK : CLD_EIO;
}

int cld_convert_data_file(const char* data_file, const char* base_cldt, const char* out_cldt) {
  std::vector<uint8_t> data, base, out;
  if (!data_file || !out_cldt) return CLD_EINVAL;
  if (read_file(data_file, &data) != CLD_OK) return CLD_EINVAL;
  const std::string bp = base_cldt ? base_cldt : default_tables_path();
  if (read_file(bp.c_str(), &base) != CLD_OK) return CLD_EINVAL;
  std::string err;
  if (cld::cld2_data_to_cldt(data.data(), data.size(), base.data(), base.size(), &out, &err) != 0) {
    fprintf(stderr, "cld_mi355x: %s: %s\n", data_file, err.c_str());
    return CLD_EINVAL;
  }
  HostTables check;   // the result must be a blob the runtime accepts
  check.blob = out;
  if (parse_tables(&check, out_cldt) != CLD_OK) return CLD_EINVAL;
  FILE* f = fopen(out_cldt, "wb");
  if (!f) return CLD_EINVAL;
  size_t w = fwrite(out.data(), 1, out.size(), f);
  return (fclose(f) == 0 && w == out.size()) ? CLD_OK : CLD_EIO;
}

// wrapper.cc:7-16.  One document through cld_detect_batch: concurrent
// callers are coalesced there (run_coalesced) into micro-batches, and a batch
// of short documents takes run_tiny (one upload, one k_wave launch, one
// download).
//
// Failures.  The reference has no error channel here and neither does
// wrapper.h, so:
//  * a document the kernels could not score (CLD_EIO: marked
//    CLD_LANG_FAILED after the batch path's own retry) gets the reference's
//    answer for "no language", UNKNOWN -> "en" (compact_lang_det.cc:91-93),
//    with a line on stderr -- one document never costs the process;
//  * no usable GPU or tables at the first call, or a device error (CLD_EFAULT,
//    CLD_ENOMEM, ...), aborts with a message: answering "en" to every caller
//    of a broken GPU would turn a deployment fault into confident wrong
//    answers (a service checks cld_init() at start).
const char* detect_language(const char* text) {
  if (cld_init(nullptr, 0) != CLD_OK) {
    fprintf(stderr, "cld_mi355x: detect_language: GPU runtime unavailable\n");
    abort();
  }
  const char* t = text ? text : "";
  const uint64_t offs[2] = {0, (uint64_t)strlen(t)};
  cld_result res{};
  int rc;
  bool queued = false;
  {
    std::shared_lock<std::shared_mutex> tl(g_swap_mu);   // (the tables stay while the call is in flight)
    if (dl_queue_takes((size_t)offs[1])) {    // the per-call queue (cld_dlqueue.h)
      const int before = g_dlq.enter();
      if (before == 0 && dl_direct(t, (size_t)offs[1], &res, &rc)) {
        g_dlq.leave();                         // (no other call in flight: run it here, no handoff)
      } else {
        cld::DlReq r((const uint8_t*)t, (size_t)offs[1], &res);
        g_dlq.push(&r);
        r.wait(before < 16 ? dl_caller_spin_us() : 0);
        rc = r.rc;
      }
      queued = true;
    }
  }
  if (!queued) rc = cld_detect_batch((const uint8_t*)t, offs, 1, &res, 0);
  if (rc != CLD_OK && !(rc == CLD_EIO && res.summary_lang == CLD_LANG_FAILED)) {
    // A coalesced call returns its whole group's code: a failure of the
    // group (e.g. CLD_ENOMEM growing the pinned arena for other callers'
    // batches) is not this document's.  Redo it alone, outside the coalescer,
    // and abort only if that fails too.
    std::shared_lock<std::shared_mutex> tl(g_swap_mu);
    Picked p(pick_context());
    res = cld_result{};
    rc = run_host_shard_isolating(p.d, (const uint8_t*)t, offs, 1, &res, 0);
  }
  std::shared_lock<std::shared_mutex> tl(g_swap_mu);
  if (rc == CLD_EIO && res.summary_lang == CLD_LANG_FAILED) {
    fprintf(stderr, "cld_mi355x: detect_language: no result for a document; answering \"en\"\n");
    res.summary_lang = (uint16_t)g_tab.meta.unknown_language;
  } else if (rc != CLD_OK) {
    fprintf(stderr, "cld_mi355x: detect_language: device error %d\n", rc);
    abort();
  }
  int lang = res.summary_lang;
  if (lang == (int)g_tab.meta.unknown_language) lang = (int)g_tab.meta.english;  // compact_lang_det.cc:91-93
  if (lang < 0 || (size_t)lang >= g_tab.codes.size()) lang = (int)g_tab.meta.unknown_language;
  return (size_t)lang < g_tab.codes.size() ? g_tab.codes[lang] : "un";
}

}  // extern "C"
