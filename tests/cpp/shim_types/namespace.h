// Test scaffold for the daemon's namespace.h.
#ifndef hyperdex_namespace_h_
#define hyperdex_namespace_h_
#define BEGIN_HYPERDEX_NAMESPACE namespace hyperdex {
#define END_HYPERDEX_NAMESPACE }
#endif
