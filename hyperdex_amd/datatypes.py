"""HyperDex data types and schema, as the hashing path sees them.

Values of enum hyperdatatype (reference include/hyperdex.h:53-102) and the
schema/attribute pair of common/schema.h:40-51 / common/attribute.h:37-49.
"""
from dataclasses import dataclass, field
from typing import List, Sequence

HYPERDATATYPE_GENERIC = 9216
HYPERDATATYPE_STRING = 9217
HYPERDATATYPE_INT64 = 9218
HYPERDATATYPE_FLOAT = 9219
HYPERDATATYPE_DOCUMENT = 9223
HYPERDATATYPE_LIST_GENERIC = 9280
HYPERDATATYPE_LIST_STRING = 9281
HYPERDATATYPE_LIST_INT64 = 9282
HYPERDATATYPE_LIST_FLOAT = 9283
HYPERDATATYPE_SET_GENERIC = 9344
HYPERDATATYPE_SET_STRING = 9345
HYPERDATATYPE_SET_INT64 = 9346
HYPERDATATYPE_SET_FLOAT = 9347
HYPERDATATYPE_MAP_GENERIC = 9408
HYPERDATATYPE_MAP_STRING_KEYONLY = 9416
HYPERDATATYPE_MAP_STRING_STRING = 9417
HYPERDATATYPE_MAP_STRING_INT64 = 9418
HYPERDATATYPE_MAP_STRING_FLOAT = 9419
HYPERDATATYPE_MAP_INT64_KEYONLY = 9424
HYPERDATATYPE_MAP_INT64_STRING = 9425
HYPERDATATYPE_MAP_INT64_INT64 = 9426
HYPERDATATYPE_MAP_INT64_FLOAT = 9427
HYPERDATATYPE_MAP_FLOAT_KEYONLY = 9432
HYPERDATATYPE_MAP_FLOAT_STRING = 9433
HYPERDATATYPE_MAP_FLOAT_INT64 = 9434
HYPERDATATYPE_MAP_FLOAT_FLOAT = 9435
HYPERDATATYPE_TIMESTAMP_GENERIC = 9472
HYPERDATATYPE_TIMESTAMP_SECOND = 9473
HYPERDATATYPE_TIMESTAMP_MINUTE = 9474
HYPERDATATYPE_TIMESTAMP_HOUR = 9475
HYPERDATATYPE_TIMESTAMP_DAY = 9476
HYPERDATATYPE_TIMESTAMP_WEEK = 9477
HYPERDATATYPE_TIMESTAMP_MONTH = 9478
HYPERDATATYPE_MACAROON_SECRET = 9664
HYPERDATATYPE_GARBAGE = 9727

TIMESTAMPS = tuple(range(HYPERDATATYPE_TIMESTAMP_SECOND, HYPERDATATYPE_TIMESTAMP_MONTH + 1))
NUMERIC = (HYPERDATATYPE_INT64, HYPERDATATYPE_FLOAT) + TIMESTAMPS
HASHABLE = (HYPERDATATYPE_STRING,) + NUMERIC
# datatype_info::lookup (datatype_info.cc:72-141) returns an object for these;
# everything else is an unknown type (assert in the reference, HDX_E_BADTYPE here).
KNOWN = HASHABLE + (
    HYPERDATATYPE_DOCUMENT,
    HYPERDATATYPE_LIST_STRING, HYPERDATATYPE_LIST_INT64, HYPERDATATYPE_LIST_FLOAT,
    HYPERDATATYPE_SET_STRING, HYPERDATATYPE_SET_INT64, HYPERDATATYPE_SET_FLOAT,
    HYPERDATATYPE_MAP_STRING_STRING, HYPERDATATYPE_MAP_STRING_INT64, HYPERDATATYPE_MAP_STRING_FLOAT,
    HYPERDATATYPE_MAP_INT64_STRING, HYPERDATATYPE_MAP_INT64_INT64, HYPERDATATYPE_MAP_INT64_FLOAT,
    HYPERDATATYPE_MAP_FLOAT_STRING, HYPERDATATYPE_MAP_FLOAT_INT64, HYPERDATATYPE_MAP_FLOAT_FLOAT,
    HYPERDATATYPE_MACAROON_SECRET,
)


@dataclass(frozen=True)
class Attribute:
    """common/attribute.h:37-49."""
    name: str
    type: int


@dataclass(frozen=True)
class Schema:
    """common/schema.h:40-51: attrs[0] is the key."""
    attrs: Sequence[Attribute] = field(default_factory=tuple)
    authorization: bool = False

    @property
    def attrs_sz(self) -> int:
        return len(self.attrs)

    def types(self) -> List[int]:
        return [a.type for a in self.attrs]

    def lookup_attr(self, name: str) -> int:
        """common/schema.cc: index of `name`, or attrs_sz when absent."""
        for i, a in enumerate(self.attrs):
            if a.name == name:
                return i
        return self.attrs_sz

    @staticmethod
    def of(*types: int) -> "Schema":
        return Schema(tuple(Attribute("k" if i == 0 else "a%d" % i, t) for i, t in enumerate(types)))
