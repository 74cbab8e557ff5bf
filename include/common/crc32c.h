// include/common/crc32c.h -- drop-in replacement header for Consus's
// common/crc32c.h (same include guard, includes, namespace and signature).
//
// replaces: common/crc32c.h:28-44
//     uint32_t consus::crc32c(uint32_t init, const unsigned char* data, size_t n);
// The definition (consus_amd/csrc/crc32c_dropin.cc) is compiled into the
// executable, as common/crc32c.cc is (Makefile.am:146), and forwards to the
// MI355X engine's C ABI (include/consus_crc32c.h, libconsus_crc32c.so).
// As in the reference, the declaration sits in the hidden-visibility consus
// namespace of namespace.h (namespace.h:4-5), whichever file includes it first.
#ifndef consus_common_crc32c_h_
#define consus_common_crc32c_h_

// C
#include <stdint.h>
#include <stdlib.h>

// consus
#include "namespace.h"

BEGIN_CONSUS_NAMESPACE

uint32_t
crc32c(uint32_t init, const unsigned char* data, size_t n);

END_CONSUS_NAMESPACE

#endif // consus_common_crc32c_h_
