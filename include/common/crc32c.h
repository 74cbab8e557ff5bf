// include/common/crc32c.h -- drop-in replacement header for Consus's
// common/crc32c.h (same include guard, same namespace, same signature).
//
// replaces: common/crc32c.h:40-41
//     uint32_t consus::crc32c(uint32_t init, const unsigned char* data, size_t n);
// The definition (consus_amd/csrc/crc32c_dropin.cc, linked into
// libconsus_crc32c.so) forwards to the MI355X engine (include/consus_crc32c.h).
// Consus declares the namespace hidden (namespace.h:4-5); so does this header
// when BEGIN_CONSUS_NAMESPACE is available, and the engine library provides a
// hidden-visibility definition for in-tree linking plus the exported C ABI.
#ifndef consus_common_crc32c_h_
#define consus_common_crc32c_h_

// C
#include <stdint.h>
#include <stdlib.h>

#ifdef BEGIN_CONSUS_NAMESPACE
BEGIN_CONSUS_NAMESPACE
#else
namespace consus {
#endif

uint32_t
crc32c(uint32_t init, const unsigned char* data, size_t n);

#ifdef END_CONSUS_NAMESPACE
END_CONSUS_NAMESPACE
#else
}
#endif

#endif // consus_common_crc32c_h_
