"""ipls -- MI355X-native IPLS gradient-partition aggregation (host side).

The arithmetic runs in hand-written gfx950 HIP kernels inside
``ipls-java-api_amd/lib/libipls_agg.so`` behind the C-ABI of
``include/ipls_agg.h``; this package is the Python twin of the Java/JNI
binding plus the Middleware wire codec.
"""
from ._native import (  # noqa: F401
    ALL_PARTITIONS, DEV_BE, DEV_F64, DEV_TEXT, HOST_BE, HOST_BE_CANON, HOST_F64, HOST_FRAME, HOST_PAIR,
    HOST_TEXT, KERNEL_FOLD1, KERNEL_REDUCE, KERNEL_REDUCE_SCALAR, KERNEL_ROUND, SHAPE_BIG, SHAPE_HALF, SHAPE_MID,
    SHAPE_SMALL, START_ACCUM, START_FIRST, START_ZERO, TGT_AGG, TGT_FUTURE, TGT_REP, TGT_WADDR, TGT_WEIGHTS,
    IplsError, build_info, lib,
)
from .aggregator import (  # noqa: F401
    Aggregator, DeviceBuffer, PinnedBuffer, checksum_dev, encode_secure, frame_encode, frame_parse, java_pair_hash,
    pair_encode, pair_parse, shard_plan, synth_fill,
)

SEED = 0x1B5_2026  # synthetic workload seed
