// extract_cld2_tables.cc -- one-shot DATA extractor (build tool, not product).
//
// Links the reference's *generated data* translation units (the CLD2 scoring
// tables, UTF-8 state machines and language/script maps that
// /root/reference/cld2/internal/compile_libs.sh:30-40 links into libcld2.so)
// and serialises every member the DetectLanguage hot path reads into one
// little-endian "CLDT" blob (format: language-detector_amd/csrc/cldt_format.h,
// DESIGN.md section 3).  No reference *code* is linked: only data TUs plus the
// header-only tables (utf8*.h, cldutil_shared.h kLgProbV2Tbl) and the three
// tiny lookup functions of lang_script.cc (LanguageCloseSet etc.), which are
// evaluated here once and stored as tables.
//
// The quadgram table (cld2_generated_quadchrome_2.cc) is a MISSING blob in
// the reference (/root/reference/.MISSING_LARGE_BLOBS:5); this tool therefore
// writes the QUAD/QUAD2 sections as absent.  tools/synth_quad.py appends the
// synthetic quadgram table.
//
// Build recipe: oracle/tablegen/Makefile  (outputs only into oracle/_ref/).

#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <vector>
#include <string>

#include "integral_types.h"
#include "cld2tablesummary.h"
#include "utf8statetable.h"
#include "cldutil_shared.h"        // kLgProbV2Tbl (header static)
#include "lang_script.h"
#include "generated_language.h"
#include "generated_ulscript.h"
#include "utf8prop_lettermarkscriptnum.h"
#include "utf8repl_lettermarklower.h"
#include "utf8scannot_lettermarkspecial.h"

namespace CLD2 {
extern const UTF8PropObj cld_generated_CjkUni_obj;
extern const CLD2TableSummary kCjkCompat_obj;
extern const CLD2TableSummary kCjkDeltaBi_obj;
extern const CLD2TableSummary kDistinctBiTable_obj;
extern const CLD2TableSummary kDeltaOcta_obj;
extern const CLD2TableSummary kDistinctOcta_obj;
extern const short kAvgDeltaOctaScore[];
extern const int kAvgDeltaOctaScoreSize;
extern const uint32 kCompatTableIndSize;
extern const uint32 kCjkDeltaBiIndSize;
extern const uint32 kDistinctBiTableIndSize;
extern const uint32 kDeltaOctaIndSize;
extern const uint32 kDistinctOctaIndSize;
extern const int kLanguageToPLangSize;
extern const uint8 kLanguageToPLang[];
extern const uint16 kPLangToLanguageLatn[];
extern const uint16 kPLangToLanguageOthr[];
extern const ULScriptRType kULScriptToRtype[];
extern const Language kULScriptToDefaultLang[];
extern const char* const kLanguageToCode[];
extern const char* const kLanguageToName[];
extern const char* const kULScriptToCode[];
}

using namespace CLD2;

#include "../../language-detector_amd/csrc/cldt_format.h"

static std::vector<uint8_t> g_out;
static std::vector<cldt_section> g_sec;

static void put(const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  g_out.insert(g_out.end(), b, b + n);
}
static void align16() { while (g_out.size() % 16) g_out.push_back(0); }

static void begin(uint32_t id) {
  align16();
  cldt_section s; memset(&s, 0, sizeof(s));
  s.id = id; s.offset = g_out.size();
  g_sec.push_back(s);
}
static void end() { g_sec.back().size = g_out.size() - g_sec.back().offset; }

static void put_u32(uint32_t v) { put(&v, 4); }

// UTF-8 state machine with one-byte entries.
static void emit_sm8(uint32_t id, const UTF8StateMachineObj* st,
                     size_t remap_n, size_t remap_str_n, bool has_fast) {
  begin(id);
  cldt_sm_header h; memset(&h, 0, sizeof(h));
  h.state0 = st->state0; h.state0_size = st->state0_size;
  h.total_size = st->total_size; h.entry_shift = st->entry_shift;
  h.bytes_per_entry = 1; h.losub = st->losub; h.hiadd = st->hiadd;
  h.n_remap = (uint32_t)remap_n; h.n_remap_string = (uint32_t)remap_str_n;
  h.has_fast = has_fast ? 1 : 0;
  put(&h, sizeof(h));
  put(st->state_table, st->total_size);
  align16();
  for (size_t i = 0; i < remap_n; ++i) {
    uint8_t e[4] = {st->remap_base[i].delete_bytes, st->remap_base[i].add_bytes,
                    (uint8_t)(st->remap_base[i].bytes_offset & 0xff),
                    (uint8_t)(st->remap_base[i].bytes_offset >> 8)};
    put(e, 4);
  }
  put(st->remap_string, remap_str_n);
  align16();
  if (has_fast) put(st->fast_state, 256);
  end();
}

static void emit_sm16(uint32_t id, const UTF8StateMachineObj_2* st) {
  begin(id);
  cldt_sm_header h; memset(&h, 0, sizeof(h));
  h.state0 = st->state0; h.state0_size = st->state0_size;
  h.total_size = st->total_size; h.entry_shift = st->entry_shift;
  h.bytes_per_entry = 2; h.losub = st->losub; h.hiadd = st->hiadd;
  put(&h, sizeof(h));
  put(st->state_table, (size_t)st->total_size * 2);
  end();
}

static void emit_summary(uint32_t id, const CLD2TableSummary* t, uint32_t n_ind) {
  begin(id);
  cldt_table_header h; memset(&h, 0, sizeof(h));
  h.size_one = t->kCLDTableSizeOne; h.size = t->kCLDTableSize;
  h.key_mask = t->kCLDTableKeyMask; h.build_date = t->kCLDTableBuildDate;
  h.n_ind = n_ind;
  // Tables declared with size 0 still allocate one (unused) bucket
  // (cld2_generated_deltaoctachrome.cc:4603-4611); store max(size,1).
  h.n_buckets_stored = t->kCLDTableSize ? t->kCLDTableSize : 1;
  put(&h, sizeof(h));
  put(t->kCLDTable, (size_t)h.n_buckets_stored * 16);
  put(t->kCLDTableInd, (size_t)n_ind * 4);
  // Sanity: every indirect referenced by a bucket must be inside the array
  uint32_t maxind = 0;
  for (uint32_t b = 0; b < h.n_buckets_stored; ++b)
    for (int k = 0; k < 4; ++k) {
      uint32_t kv = t->kCLDTable[b].keyvalue[k];
      if (kv == 0) continue;
      uint32_t ind = kv & ~t->kCLDTableKeyMask;
      uint32_t need = ind < t->kCLDTableSizeOne ? ind + 1
                      : ind + (ind - t->kCLDTableSizeOne) + 2;
      if (need > maxind) maxind = need;
    }
  if (maxind > n_ind) {
    fprintf(stderr, "table %u: indirect %u beyond ind array %u\n", id, maxind, n_ind);
    exit(2);
  }
  end();
}

// The 8-byte fast paths of UTF8GenericScan (utf8statetable.cc:486-507) skip
// bytes without consulting the state table.  The restatements run the plain
// byte-at-a-time loop, which is equivalent iff every skippable byte maps
// state0 -> state0 with no exit.  Verify that here, once, on the real table.
static void check_fast_equiv(const char* name, const UTF8StateMachineObj* st) {
  const uint8* tbl0 = &st->state_table[st->state0];
  uint8_t lo = st->losub & 0xff, hi = st->hiadd & 0xff;
  for (int c = 0; c < 256; ++c) {
    bool range = (c >= lo) && (c + hi < 0x80);
    bool fast0 = st->fast_state && st->fast_state[c] == 0;
    if ((range || fast0) && tbl0[c] != 0) {
      fprintf(stderr, "%s: byte %02x skippable by fast path but state0 entry %d\n",
              name, c, tbl0[c]);
      exit(3);
    }
  }
}

int main(int argc, char** argv) {
  if (argc != 2) { fprintf(stderr, "usage: %s out.cldt\n", argv[0]); return 1; }

  check_fast_equiv("scannot", &utf8scannot_lettermarkspecial_obj);

  // Header placeholder
  cldt_file_header fh; memset(&fh, 0, sizeof(fh));
  put(&fh, sizeof(fh));

  begin(CLDT_META);
  cldt_meta m; memset(&m, 0, sizeof(m));
  m.num_languages = NUM_LANGUAGES; m.num_ulscripts = NUM_ULSCRIPTS;
  m.lang_to_plang_size = kLanguageToPLangSize;
  m.english = ENGLISH; m.unknown_language = UNKNOWN_LANGUAGE;
  m.tg_unknown_language = TG_UNKNOWN_LANGUAGE; m.chinese = CHINESE;
  m.chinese_t = CHINESE_T; m.french = FRENCH; m.italian = ITALIAN;
  m.german = GERMAN; m.spanish = SPANISH; m.hawaiian = HAWAIIAN;
  m.ulscript_common = ULScript_Common; m.ulscript_latin = ULScript_Latin;
  m.ulscript_cyrillic = ULScript_Cyrillic; m.ulscript_arabic = ULScript_Arabic;
  m.ulscript_hani = ULScript_Hani; m.ulscript_inherited = ULScript_Inherited;
  put(&m, sizeof(m));
  end();

  emit_sm16(CLDT_SCRIPT_PROP, &utf8prop_lettermarkscriptnum_obj);
  emit_sm8(CLDT_LOWER_REPL, &utf8repl_lettermarklower_obj,
           sizeof(utf8repl_lettermarklower_remap_base) / sizeof(RemapEntry),
           sizeof(utf8repl_lettermarklower_remap_string), false);
  emit_sm8(CLDT_SCAN_NOT, &utf8scannot_lettermarkspecial_obj, 0, 0, true);
  emit_sm8(CLDT_CJK_UNI_PROP, &cld_generated_CjkUni_obj, 0, 0, false);

  emit_summary(CLDT_CJK_COMPAT, &kCjkCompat_obj, kCompatTableIndSize);
  emit_summary(CLDT_DELTA_BI, &kCjkDeltaBi_obj, kCjkDeltaBiIndSize);
  emit_summary(CLDT_DISTINCT_BI, &kDistinctBiTable_obj, kDistinctBiTableIndSize);
  emit_summary(CLDT_DELTA_OCTA, &kDeltaOcta_obj, kDeltaOctaIndSize);
  emit_summary(CLDT_DISTINCT_OCTA, &kDistinctOcta_obj, kDistinctOctaIndSize);

  begin(CLDT_EXPECTED_SCORE);
  put(kAvgDeltaOctaScore, (size_t)kAvgDeltaOctaScoreSize * 2);
  end();

  begin(CLDT_LGPROB);
  put(kLgProbV2Tbl, sizeof(kLgProbV2Tbl));
  end();

  begin(CLDT_LANG_TO_PLANG);
  put(kLanguageToPLang, kLanguageToPLangSize);
  end();
  begin(CLDT_PLANG_TO_LANG_LATN);
  put(kPLangToLanguageLatn, 512);
  end();
  begin(CLDT_PLANG_TO_LANG_OTHR);
  put(kPLangToLanguageOthr, 512);
  end();

  begin(CLDT_ULSCRIPT_RTYPE);
  for (int i = 0; i < NUM_ULSCRIPTS; ++i) { uint8_t v = kULScriptToRtype[i]; put(&v, 1); }
  end();
  begin(CLDT_ULSCRIPT_DEFAULT_LANG);
  for (int i = 0; i < NUM_ULSCRIPTS; ++i) { uint16_t v = kULScriptToDefaultLang[i]; put(&v, 2); }
  end();

  // kClosestAltLanguage (compact_lang_det_impl.cc:259-427), via closest_alt.inc
  {
    static const Language kAlt[] = {
#include "closest_alt.inc"
    };
    if (sizeof(kAlt) / sizeof(kAlt[0]) != (size_t)HAWAIIAN + 1) {
      fprintf(stderr, "closest-alt size %zu != %d\n", sizeof(kAlt) / sizeof(kAlt[0]), HAWAIIAN + 1);
      exit(4);
    }
    begin(CLDT_CLOSEST_ALT);
    for (size_t i = 0; i < sizeof(kAlt) / sizeof(kAlt[0]); ++i) {
      uint16_t v = kAlt[i]; put(&v, 2);
    }
    end();
  }

  // LanguageCloseSet (lang_script.cc:261-310) evaluated once per language.
  begin(CLDT_CLOSE_SET);
  for (int i = 0; i < NUM_LANGUAGES; ++i) {
    uint8_t v = (uint8_t)LanguageCloseSet((Language)i); put(&v, 1);
  }
  end();

  // Strings: u32 count, u32 offsets[count+1], bytes
  auto emit_strings = [](uint32_t id, const char* const* arr, int n) {
    begin(id);
    put_u32(n);
    uint32_t off = 0;
    for (int i = 0; i < n; ++i) { put_u32(off); off += strlen(arr[i]) + 1; }
    put_u32(off);
    for (int i = 0; i < n; ++i) put(arr[i], strlen(arr[i]) + 1);
    end();
  };
  emit_strings(CLDT_LANG_CODES, kLanguageToCode, NUM_LANGUAGES);
  emit_strings(CLDT_LANG_NAMES, kLanguageToName, NUM_LANGUAGES);
  emit_strings(CLDT_ULSCRIPT_CODES, kULScriptToCode, NUM_ULSCRIPTS);

  align16();
  fh.magic = CLDT_MAGIC; fh.version = CLDT_VERSION;
  fh.n_sections = (uint32_t)g_sec.size();
  fh.section_table_offset = g_out.size();
  for (auto& s : g_sec) put(&s, sizeof(s));
  memcpy(g_out.data(), &fh, sizeof(fh));

  FILE* f = fopen(argv[1], "wb");
  if (!f) { perror(argv[1]); return 1; }
  fwrite(g_out.data(), 1, g_out.size(), f);
  fclose(f);
  fprintf(stderr, "wrote %s: %zu bytes, %zu sections\n", argv[1], g_out.size(), g_sec.size());
  return 0;
}
