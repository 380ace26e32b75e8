"""CESS geometry constants the codec is built for (values from the reference chain)."""

M_BYTE = 1_048_576                      # primitives/common/src/lib.rs:56
SEGMENT_SIZE = M_BYTE * 16              # primitives/common/src/lib.rs:60
FRAGMENT_SIZE = M_BYTE * 8              # primitives/common/src/lib.rs:61
CHUNK_COUNT = 1024                      # primitives/common/src/lib.rs:62
FRAGMENT_COUNT = 3                      # runtime/src/lib.rs:1027
SEGMENT_COUNT = 1000                    # runtime/src/lib.rs:1026 (segments per file)
HASH_LEN = 64                           # Hash([u8; 64]), primitives/common/src/lib.rs:16

DATA_SHARDS = SEGMENT_SIZE // FRAGMENT_SIZE          # k = 2
PARITY_SHARDS = FRAGMENT_COUNT - DATA_SHARDS         # m = 1
# space locked per segment: SEGMENT_SIZE * 15 / 10 (c-pallets/file-bank/src/lib.rs:440)
SEGMENT_SPACE = SEGMENT_SIZE * 15 // 10
assert SEGMENT_SPACE == FRAGMENT_COUNT * FRAGMENT_SIZE

# wide-code stress geometry (BASELINE.json config 5): same 16 MiB segment, RS(32+32)
WIDE_DATA_SHARDS = 32
WIDE_PARITY_SHARDS = 32
WIDE_FRAGMENT_SIZE = SEGMENT_SIZE // WIDE_DATA_SHARDS  # 512 KiB
