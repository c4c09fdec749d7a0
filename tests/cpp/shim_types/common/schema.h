// Test scaffold for the daemon's common/schema.h + common/attribute.h +
// enum hyperdatatype (values: include/hyperdex.h of the reference).
#ifndef hyperdex_common_schema_h_
#define hyperdex_common_schema_h_
#include <stdint.h>
enum hyperdatatype {
    HYPERDATATYPE_STRING = 9217, HYPERDATATYPE_INT64 = 9218, HYPERDATATYPE_FLOAT = 9219,
    HYPERDATATYPE_LIST_STRING = 9281, HYPERDATATYPE_TIMESTAMP_SECOND = 9473,
    HYPERDATATYPE_TIMESTAMP_MONTH = 9478
};
namespace hyperdex {
struct attribute {
    const char* name;
    hyperdatatype type;
};
struct schema {
    uint16_t attrs_sz;
    const attribute* attrs;
    bool authorization;
};
}  // namespace hyperdex
#endif
