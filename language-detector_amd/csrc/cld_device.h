// cld_device.h -- device-side view of the CLDT tables and the batch result
// record.  Shared by the HIP kernels and the host runtime.
#ifndef CLD_DEVICE_H_
#define CLD_DEVICE_H_

#include <stdint.h>

// One UTF-8 state machine (utf8statetable.h:101-130)
struct DevSM {
  const uint8_t* t8;
  const uint16_t* t16;
  const uint8_t* remap;       // {del, add, off_lo, off_hi} x n_remap
  const uint8_t* rstr;
  uint32_t state0, state0_size, total, shift, n_remap, n_rstr;
};

// One CLD2TableSummary (cld2tablesummary.h:37-49)
struct DevTbl {
  const uint32_t* b;          // n_buckets x 4 keyvalues
  const uint32_t* ind;        // indirect langprobs
  const uint64_t* adds;       // per indirect entry: its langprob's three tote adds (lng::tote_adds),
                              // bit 63 set if the langprob is non-zero (k_long; built on device)
  uint32_t size_one, size, key_mask, n_ind, n_buckets;
};

// Everything DetectLanguageSummaryV2 reads, as device pointers into one
// uploaded blob plus the handful of enum values the algorithm names.
struct DevTables {
  DevSM script, lower, scan, uni;
  DevTbl compat, deltabi, distinctbi, quad, quad2, deltaocta, distinctocta;
  const int16_t* expected;
  const uint8_t* lgprob;
  const uint8_t* l2p;
  const uint16_t* p2l_latn;
  const uint16_t* p2l_othr;
  const uint8_t* rtype;
  const uint16_t* deflang;
  const uint16_t* closest;
  const uint64_t* cpt;        // per-character properties of 1-3 byte sequences (cld_long.hip, built on device)
  const uint64_t* keytab;     // per (script, key): language, close set, expected score (k_long, built on device)
  const uint8_t* close_set;
  const uint8_t* ent_names;   // HTML mode: entity name string section (CLDT_ENTITY_NAMES), or null
  const int32_t* ent_values;  //   and their code points
  const uint32_t* cp1252;     //   FixUnicodeValue below U+0100
  uint32_t n_ent;
  uint32_t n_expected, l2p_size, n_scripts, n_langs, n_closest;
  uint32_t latin, cyrillic, arabic, common, inherited;
  uint32_t unknown_lang, english, tg_unknown, french, italian, german, spanish, hawaiian;
};

#ifdef __cplusplus
extern "C" {
#endif
#include "../../include/cld_mi355x.h"
#ifdef __cplusplus
}
#endif

// Per-document status written next to the result
enum {
  CLD_ST_DONE = 0,
  CLD_ST_REQUEUE = 1,     // short kernel could not finish: k_long redoes it
  CLD_ST_ERROR = 2
};

#endif  // CLD_DEVICE_H_
