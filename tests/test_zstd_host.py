"""The ZSTD decoder of csrc/kernels/zstd_decode.h run on the host (one-lane
instantiation, ``_native.zstd_decompress_host``) against pyarrow's libzstd
on frames of every shape the format has: raw / RLE / compressed blocks,
raw / RLE / Huffman (1 and 4 streams, direct and FSE-coded weights) /
treeless literals, predefined / RLE / FSE / repeated sequence tables,
repeat offsets, multi-block frames, concatenated frames and every
compression level class. The GPU instantiation is checked on real pages in
tests/test_parquet_gpu.py; corrupt input must fail with an error code, never
crash."""
import numpy as np
import pyarrow as pa
import pytest

from igloo_amd.ops._lib import native

RNG = np.random.default_rng(0)
WORDS = ["special", "requests", "carefully", "final", "deposits", "the", "of", "x", "ironic", "pinto beans"]
CASES = {
    "empty": b"",
    "tiny": b"abc",
    "random": RNG.integers(0, 256, 200_000, dtype=np.uint8).tobytes(),
    "text": " ".join(RNG.choice(WORDS, 120_000)).encode(),
    "arange64": np.arange(200_000, dtype=np.int64).tobytes(),
    "arange32x7": (np.arange(300_000, dtype=np.int32) * 7).tobytes(),
    "zeros": bytes(700_000),
    "smallint": RNG.integers(0, 50, 400_000).astype(np.int32).tobytes(),
    "floats": RNG.normal(size=100_000).tobytes(),
    "repeats": (b"abcdefgh" * 3 + b"xyz") * 20_000,
    "far": (RNG.integers(0, 256, 40_000, dtype=np.uint8).tobytes() * 5),   # matches 40 KB back
    "mixed": b"".join(RNG.integers(0, 256, int(k), dtype=np.uint8).tobytes() + bytes(int(k))
                      for k in RNG.integers(1, 3000, 300)),
}


@pytest.mark.parametrize("level", [1, 3, 9, 19, -5])
@pytest.mark.parametrize("name", sorted(CASES))
def test_host_decoder_matches_libzstd(name, level):
    data = CASES[name]
    comp = pa.Codec("zstd", compression_level=level).compress(data, asbytes=True)
    err, out = native().zstd_decompress_host(comp, len(data))
    assert err == 0 and out == data


def test_concatenated_frames():
    a, b = CASES["text"][:50_000], CASES["smallint"][:70_000]
    c = pa.Codec("zstd")
    err, out = native().zstd_decompress_host(c.compress(a, asbytes=True) + c.compress(b, asbytes=True), len(a) + len(b))
    assert err == 0 and out == a + b


def test_corrupt_input_reports_an_error():
    data = CASES["text"][:100_000]
    comp = bytearray(pa.Codec("zstd", compression_level=3).compress(data, asbytes=True))
    N = native()
    assert N.zstd_decompress_host(b"not zstd at all", 10)[0] == 20
    assert N.zstd_decompress_host(bytes(comp), len(data) + 1)[0] != 0           # size mismatch
    rng = np.random.default_rng(5)
    for _ in range(200):                                                        # flipped bytes: error or garbage,
        bad = bytearray(comp)                                                    # never a crash
        for pos in rng.integers(4, len(bad), 3):
            bad[pos] ^= int(rng.integers(1, 256))
        N.zstd_decompress_host(bytes(bad), len(data))
    assert N.zstd_decompress_host(bytes(comp[: len(comp) // 2]), len(data))[0] != 0
