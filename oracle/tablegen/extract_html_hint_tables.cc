// extract_html_hint_tables.cc -- DATA extractor (build tool, not product) for
// the HTML-mode and hint tables, appended to the CLDT blob written by
// extract_cld2_tables.cc.
//
//   entities        kNameToEntity (generated_entities.cc, a data TU, linked)
//   cp1252 fix      kMapFullMicrosoft1252OrSpace (fixunicodevalue.h, header table)
//   hint tables     kCLDLangTagsHintTable1/2, kCLDTLDHintTable, kLangCodeAction,
//                   kLangCodeRemap: file-static in compact_lang_det_hint_code.cc,
//                   so this TU compiles that file where it lies (#include by
//                   path, -I$(REF)) to read them -- nothing is copied
//   encoding priors SetCLDEncodingHint probed once per Encoding value
//
// Usage: extract_html_hint_tables in.cldt out.cldt
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "compact_lang_det_hint_code.cc"   // the reference's file, for its static tables
#include "fixunicodevalue.h"
#include "../public/encodings.h"

namespace CLD2 {
extern const int kNameToEntitySize;
extern const CharIntPair kNameToEntity[];
}  // namespace CLD2

#include "../../language-detector_amd/csrc/cldt_format.h"

using namespace CLD2;

static std::vector<uint8_t> g_in, g_out;
static std::vector<cldt_section> g_sec;

static void put(const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  g_out.insert(g_out.end(), b, b + n);
}
static void align16() { while (g_out.size() % 16) g_out.push_back(0); }
static void begin(uint32_t id) {
  align16();
  cldt_section s;
  memset(&s, 0, sizeof(s));
  s.id = id;
  s.offset = g_out.size();
  g_sec.push_back(s);
}
static void end() { g_sec.back().size = g_out.size() - g_sec.back().offset; }
static void put_u32(uint32_t v) { put(&v, 4); }

template <class E, class K, class C>
static void emit_hint(uint32_t id, const E* tbl, int n, K key, C code) {
  begin(id);
  put_u32(n);
  std::string pool;
  for (int i = 0; i < n; ++i) {
    cldt_hint_entry e;
    e.key_off = (uint32_t)pool.size();
    pool.append(key(tbl[i]));
    pool.push_back(0);
    const char* c = code(tbl[i]);
    if (c) {
      e.code_off = (uint32_t)pool.size();
      pool.append(c);
      pool.push_back(0);
    } else {
      e.code_off = 0xFFFFFFFFu;
    }
    e.prior1 = tbl[i].onelangprior1;
    e.prior2 = tbl[i].onelangprior2;
    put(&e, sizeof(e));
  }
  put(pool.data(), pool.size());
  end();
}

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: %s in.cldt out.cldt\n", argv[0]); return 1; }
  FILE* f = fopen(argv[1], "rb");
  if (!f) { perror(argv[1]); return 1; }
  fseek(f, 0, SEEK_END);
  g_in.resize(ftell(f));
  fseek(f, 0, SEEK_SET);
  if (fread(g_in.data(), 1, g_in.size(), f) != g_in.size()) return 1;
  fclose(f);
  // copy every section of the input blob
  cldt_file_header fh;
  memcpy(&fh, g_in.data(), sizeof(fh));
  put(&fh, sizeof(fh));
  const cldt_section* in_sec = (const cldt_section*)(g_in.data() + fh.section_table_offset);
  for (uint32_t i = 0; i < fh.n_sections; ++i) {
    begin(in_sec[i].id);
    put(g_in.data() + in_sec[i].offset, in_sec[i].size);
    end();
  }

  begin(CLDT_ENTITY_NAMES);
  put_u32(kNameToEntitySize);
  {
    uint32_t off = 0;
    for (int i = 0; i < kNameToEntitySize; ++i) { put_u32(off); off += strlen(kNameToEntity[i].s) + 1; }
    put_u32(off);
    for (int i = 0; i < kNameToEntitySize; ++i) put(kNameToEntity[i].s, strlen(kNameToEntity[i].s) + 1);
  }
  end();
  begin(CLDT_ENTITY_VALUES);
  for (int i = 0; i < kNameToEntitySize; ++i) { int32_t v = kNameToEntity[i].i; put(&v, 4); }
  end();
  begin(CLDT_CP1252_FIX);
  for (int i = 0; i < 256; ++i) put_u32((uint32_t)kMapFullMicrosoft1252OrSpace[i]);
  end();

  emit_hint(CLDT_HINT_LANGTAG1, kCLDLangTagsHintTable1, kCLDTable1Size,
            [](const LangTagLookup& e) { return e.langtag; }, [](const LangTagLookup& e) { return e.langcode; });
  emit_hint(CLDT_HINT_LANGTAG2, kCLDLangTagsHintTable2, kCLDTable2Size,
            [](const LangTagLookup& e) { return e.langtag; }, [](const LangTagLookup& e) { return e.langcode; });
  emit_hint(CLDT_HINT_TLD, kCLDTLDHintTable, kCLDTable3Size, [](const TLDLookup& e) { return e.tld; },
            [](const TLDLookup&) { return (const char*)nullptr; });
  begin(CLDT_HINT_CODE_ACTION);
  put(kLangCodeAction, 256);
  end();
  begin(CLDT_HINT_CODE_REMAP);
  put(kLangCodeRemap, 256);
  end();
  begin(CLDT_HINT_ENCODING);
  for (int e = 0; e < NUM_ENCODINGS; ++e) {
    CLDLangPriors lp;
    InitCLDLangPriors(&lp);
    SetCLDEncodingHint((Encoding)e, &lp);
    int16_t v = lp.n ? lp.prior[0] : 0;
    put(&v, 2);
  }
  end();

  align16();
  fh.n_sections = (uint32_t)g_sec.size();
  fh.section_table_offset = g_out.size();
  for (auto& s : g_sec) put(&s, sizeof(s));
  memcpy(g_out.data(), &fh, sizeof(fh));
  f = fopen(argv[2], "wb");
  if (!f) { perror(argv[2]); return 1; }
  fwrite(g_out.data(), 1, g_out.size(), f);
  fclose(f);
  fprintf(stderr, "wrote %s: %zu bytes, %zu sections (entities %d, langtags %d/%d, tlds %d)\n", argv[2],
          g_out.size(), g_sec.size(), kNameToEntitySize, kCLDTable1Size, kCLDTable2Size, kCLDTable3Size);
  return 0;
}
