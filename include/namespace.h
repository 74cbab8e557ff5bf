// include/namespace.h -- the namespace macros of Consus's namespace.h
// (namespace.h:4-5), restated so that include/common/crc32c.h can include
// "namespace.h" exactly as the reference header does (common/crc32c.h:33-35).
// Same include guard: inside the Consus tree its own namespace.h is found
// first (-I$(top_srcdir)) and this one is never read.
#ifndef consus_namespace_h_
#define consus_namespace_h_

#define BEGIN_CONSUS_NAMESPACE namespace consus __attribute__((visibility("hidden"))) {
#define END_CONSUS_NAMESPACE }

#endif  // consus_namespace_h_
