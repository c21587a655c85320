// cld_dynamic_data.h -- CLD2 dynamic data file -> CLDT blob (host only).
#ifndef CLD_DYNAMIC_DATA_H_
#define CLD_DYNAMIC_DATA_H_

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace cld {
// Builds a CLDT blob from a "cld2_data_file00" image (cld2_dynamic_data.h:22-147)
// and a base CLDT blob that supplies the sections the data file does not carry.
// Returns 0 or CLD_EINVAL (-22) with a reason in *err.
int cld2_data_to_cldt(const uint8_t* data, size_t len, const uint8_t* base, size_t base_len,
                      std::vector<uint8_t>* out, std::string* err);
}  // namespace cld

#endif  // CLD_DYNAMIC_DATA_H_
