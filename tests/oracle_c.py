"""Re-export of the C-oracle loader for the tests."""
from oracle.c_oracle import c_encode, c_sha256_hex, load_c_oracle, ptrs  # noqa: F401
