// dynload.cc -- TEST INFRASTRUCTURE ONLY.  Loads a cld2_data_file00 through
// the reference's own loader (CLD2DynamicDataLoader::loadDataFile,
// cld2_dynamic_data_loader.cc:164-258, compiled where it lies by Makefile) and
// prints what it reconstructed, so tests/test_dynamic_data.py can check that
// the files tools/cld2_data_file.py writes are read back by the reference into
// exactly the tables they were written from.
//   dynload <file> <n_expected_shorts> <n_ind_0> ... <n_ind_6>
// Output: one JSON object; byte blocks as FNV-1a 64 hex digests.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cld2_dynamic_data.h"
#include "cld2_dynamic_data_loader.h"
#include "scoreonescriptspan.h"

static uint64_t fnv(const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
  return h;
}

int main(int argc, char** argv) {
  if (argc < 10) { fprintf(stderr, "usage: dynload <file> <n_expected> <n_ind x7>\n"); return 2; }
  void* addr = nullptr;
  uint32_t len = 0;
  CLD2::ScoringTables* t = CLD2DynamicDataLoader::loadDataFile(argv[1], &addr, &len);
  if (!t) { printf("{\"loaded\": false}\n"); return 0; }
  const CLD2::UTF8PropObj* u = t->unigram_obj;
  printf("{\"loaded\": true, \"length\": %u, \"unigram\": {\"state0\": %u, \"state0_size\": %u, \"total_size\": %u, "
         "\"max_expand\": %d, \"entry_shift\": %d, \"bytes_per_entry\": %d, \"losub\": %u, \"hiadd\": %u, "
         "\"state_table\": \"%016llx\", \"remap_string\": \"%016llx\", \"fast_state\": %s}",
         len, u->state0, u->state0_size, u->total_size, u->max_expand, u->entry_shift, u->bytes_per_entry,
         u->losub, u->hiadd, (unsigned long long)fnv(u->state_table, (size_t)u->total_size * u->bytes_per_entry),
         (unsigned long long)fnv(u->remap_string, strlen((const char*)u->remap_string) + 1),
         u->fast_state ? "true" : "false");
  printf(", \"expected\": \"%016llx\"", (unsigned long long)fnv(t->kExpectedScore, 2ull * atoi(argv[2])));
  const CLD2::CLD2TableSummary* s[7] = {t->unigram_compat_obj, t->deltabi_obj, t->distinctbi_obj,
                                        t->quadgram_obj, t->quadgram_obj2, t->deltaocta_obj,
                                        t->distinctocta_obj};
  printf(", \"tables\": [");
  for (int i = 0; i < 7; ++i) {
    printf("%s{\"size_one\": %u, \"size\": %u, \"key_mask\": %u, \"build_date\": %u, \"buckets\": \"%016llx\", "
           "\"ind\": \"%016llx\", \"recognized\": \"%s\"}",
           i ? ", " : "", s[i]->kCLDTableSizeOne, s[i]->kCLDTableSize, s[i]->kCLDTableKeyMask,
           s[i]->kCLDTableBuildDate, (unsigned long long)fnv(s[i]->kCLDTable, 16ull * s[i]->kCLDTableSize),
           (unsigned long long)fnv(s[i]->kCLDTableInd, 4ull * atoi(argv[3 + i])), s[i]->kRecognizedLangScripts);
  }
  printf("]}\n");
  CLD2DynamicDataLoader::unloadDataFile(&t, &addr, &len);
  return 0;
}
