// consus_amd/csrc/crc32c_dropin.cc -- definition behind include/common/crc32c.h.
//
// replaces: common/crc32c.cc:122-126
//     uint32_t consus::crc32c(uint32_t init, const unsigned char* data, size_t n)
// Same signature and results; the checksum is computed by the MI355X engine
// (include/consus_crc32c.h).  Total, as the reference is: mi_crc32c completes
// an engine failure on the engine's CPU path and counts it (mi_crc32c_stats).
#include "../../include/common/crc32c.h"

#include "../../include/consus_crc32c.h"

uint32_t consus::crc32c(uint32_t init, const unsigned char* data, size_t n)
{
    return mi_crc32c(init, data, n);
}
