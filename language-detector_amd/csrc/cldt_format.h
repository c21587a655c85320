// cldt_format.h -- on-disk layout of the CLDT table blob.
//
// One little-endian file holds every read-only table the CLD2 DetectLanguage
// hot path consults (the reference's ScoringTables struct,
// /root/reference/cld2/internal/scoreonescriptspan.h:100-114, plus the UTF-8
// state machines and the language/script maps).  Loaded once per process and
// uploaded once per GPU.  Plain C so the C oracle, the host runtime and the
// table tools share it.
#ifndef CLDT_FORMAT_H_
#define CLDT_FORMAT_H_

#include <stdint.h>

#define CLDT_MAGIC 0x54444C43u   /* "CLDT" */
#define CLDT_VERSION 1u

enum cldt_section_id {
  CLDT_META = 1,
  CLDT_SCRIPT_PROP = 2,          /* utf8prop_lettermarkscriptnum (u16 entries) */
  CLDT_LOWER_REPL = 3,           /* utf8repl_lettermarklower (u8 + remap)      */
  CLDT_SCAN_NOT = 4,             /* utf8scannot_lettermarkspecial (u8)         */
  CLDT_CJK_UNI_PROP = 5,         /* cld_generated_CjkUni_obj (u8, BigOneByte)  */
  CLDT_CJK_COMPAT = 10,          /* CLD2TableSummary sections ...              */
  CLDT_DELTA_BI = 11,
  CLDT_DISTINCT_BI = 12,
  CLDT_QUAD = 13,
  CLDT_QUAD2 = 14,
  CLDT_DELTA_OCTA = 15,
  CLDT_DISTINCT_OCTA = 16,
  CLDT_EXPECTED_SCORE = 20,      /* int16[num_languages*4]                      */
  CLDT_LGPROB = 21,              /* uint8[240*8] kLgProbV2Tbl                   */
  CLDT_LANG_TO_PLANG = 22,       /* uint8[lang_to_plang_size]                   */
  CLDT_PLANG_TO_LANG_LATN = 23,  /* uint16[256]                                 */
  CLDT_PLANG_TO_LANG_OTHR = 24,  /* uint16[256]                                 */
  CLDT_ULSCRIPT_RTYPE = 25,      /* uint8[num_ulscripts]                        */
  CLDT_ULSCRIPT_DEFAULT_LANG = 26, /* uint16[num_ulscripts]                     */
  CLDT_CLOSEST_ALT = 27,         /* uint16[hawaiian+1]                          */
  CLDT_CLOSE_SET = 28,           /* uint8[num_languages]                        */
  CLDT_LANG_CODES = 29,          /* string table                                */
  CLDT_LANG_NAMES = 30,
  CLDT_ULSCRIPT_CODES = 31,
  /* HTML mode (getonescriptspan.cc:150-541) and hints (compact_lang_det_hint_code.cc);
   * optional: a blob without them supports plain text without hints only */
  CLDT_ENTITY_NAMES = 32,        /* string table, sorted (generated_entities.cc) */
  CLDT_ENTITY_VALUES = 33,       /* int32[n] code points                        */
  CLDT_CP1252_FIX = 34,          /* uint32[256] FixUnicodeValue below U+0100    */
  CLDT_HINT_LANGTAG1 = 35,       /* cldt_hint_entry[n] + string pool, sorted    */
  CLDT_HINT_LANGTAG2 = 36,
  CLDT_HINT_TLD = 37,
  CLDT_HINT_CODE_ACTION = 38,    /* uint8[256] language-attribute scanner       */
  CLDT_HINT_CODE_REMAP = 39,     /* uint8[256]                                  */
  CLDT_HINT_ENCODING = 41,       /* int16[n_encodings] prior per Encoding (0: none) */
  CLDT_PROVENANCE = 40           /* free text: how each section was produced    */
};

typedef struct {
  uint32_t magic, version, n_sections, reserved;
  uint64_t section_table_offset;
  uint64_t reserved2;
} cldt_file_header;

typedef struct {
  uint32_t id, reserved;
  uint64_t offset, size;
  uint64_t reserved2;
} cldt_section;

typedef struct {
  uint32_t num_languages, num_ulscripts, lang_to_plang_size;
  uint32_t english, unknown_language, tg_unknown_language, chinese, chinese_t;
  uint32_t french, italian, german, spanish, hawaiian;
  uint32_t ulscript_common, ulscript_latin, ulscript_cyrillic, ulscript_arabic;
  uint32_t ulscript_hani, ulscript_inherited;
  uint32_t reserved[13];
} cldt_meta;

/* UTF-8 state machine (utf8statetable.h:101-114).  Followed by the table
 * (total_size entries of bytes_per_entry), pad16, n_remap 4-byte remap
 * entries {del, add, off_lo, off_hi}, n_remap_string bytes, pad16, then
 * 256 fast-state bytes if has_fast. */
typedef struct {
  uint32_t state0, state0_size, total_size, entry_shift;
  uint32_t bytes_per_entry, losub, hiadd, n_remap;
  uint32_t n_remap_string, has_fast, reserved[2];
} cldt_sm_header;

/* CLD2TableSummary (cld2tablesummary.h:37-49).  Followed by
 * n_buckets_stored 16-byte buckets and n_ind uint32 indirect langprobs. */
typedef struct {
  uint32_t size_one, size, key_mask, build_date;
  uint32_t n_ind, n_buckets_stored, reserved[2];
} cldt_table_header;

/* Hint lookup tables (LangTagLookup / TLDLookup, compact_lang_det_hint_code.cc):
 * u32 n, then n entries, then the string pool; offsets are into the pool,
 * code_off = 0xFFFFFFFF when the table has no language-code column.  A prior
 * is OneCLDLangPrior: (weight << 10) + Language, int16. */
typedef struct {
  uint32_t key_off, code_off;
  int16_t prior1, prior2;
} cldt_hint_entry;

#endif  /* CLDT_FORMAT_H_ */
