"""hyperdex_amd — MI355X-native hyperspace attribute hashing.

Drop-in for HyperDex's per-object attribute hashing (common/hash.{h,cc},
cityhash/city.cc, common/ordered_encoding.cc, common/datatype_*.cc::hash):
the hash runs as hand-written gfx950 HIP kernels in libhdxhash.so behind the
C-ABI of include/hdxhash.h.  This package is the Python host side; the C++
host side is include/hyperdex_amd/hash.h.
"""
from ._lib import HdxError, lib  # noqa: F401
from .datatypes import *  # noqa: F401,F403
from .datatypes import Attribute, Schema  # noqa: F401
from .hashing import (hash, hash_batch, hash_batch_host, hash_encoded, hash_encoded_regions, hash_batch_regions,  # noqa: F401
                      hash_key, hash_object, hashable, schema_check, init_mask, device_set, shutdown,
                      hash_batch_device_multi, hash_batch_regions_host, hash_encoded_host,
                      hash_encoded_host_status, hash_batch_regions_device_multi)
from .regions import PointLeaderAbort, PointLeaders, RegionTable, lookup_region  # noqa: F401
from .index import index_encode, index_key_size, search_regions, search_space  # noqa: F401
from .batcher import Batcher  # noqa: F401

__all__ = ["HdxError", "Attribute", "Schema", "hash", "hash_key", "hash_object", "hash_batch",
           "hash_batch_host", "hash_encoded", "hash_encoded_regions", "hash_batch_regions", "hash_batch_regions_host",
           "hash_encoded_host", "hash_encoded_host_status", "hash_batch_device_multi", "hash_batch_regions_device_multi",
           "init_mask", "device_set", "shutdown", "hashable", "schema_check", "RegionTable",
           "lookup_region", "PointLeaders", "PointLeaderAbort", "index_encode", "index_key_size", "search_regions", "search_space", "Batcher", "lib"]
