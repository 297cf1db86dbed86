"""Generate tests/golden/chacha20_kat.json with the container's openssl.

openssl's ChaCha20 (RFC 7539: 32-bit counter + 96-bit nonce) and rand_chacha's
layout (64-bit counter in words 12-13, 64-bit stream in 14-15) coincide when the
stream is 0 and the block counter is below 2^32, so keystream block `c` under key
`k` is `openssl enc -chacha20 -K <k> -iv <c as 4 LE bytes || 12 zero bytes>`
applied to 64 zero bytes. Keys are the PCG32 fills of rand_core's
seed_from_u64 (restated in oracle/rabia_ref.py), stored as their LE bytes, so the
fixture pins the ChaCha core AND the key-word byte order at 20 rounds.
Run: python tools/make_chacha_kat.py   (needs openssl on PATH; no network)
"""
import json
import os
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rabia_ref as R  # noqa: E402


def openssl_block(key_bytes: bytes, counter: int) -> bytes:
    iv = struct.pack("<I", counter) + bytes(12)
    out = subprocess.run(
        ["openssl", "enc", "-chacha20", "-K", key_bytes.hex(), "-iv", iv.hex()],
        input=bytes(64), capture_output=True, check=True).stdout
    assert len(out) == 64
    return out


def main():
    cases = []
    keys = {"zero": [0] * 8}
    for seed in (0, 1, 42, 0xFFFFFFFFFFFFFFFF):
        keys[f"seed_from_u64({seed})"] = R.seed_from_u64(seed)
    for name, key in keys.items():
        kb = struct.pack("<8I", *key)
        for counter in (0, 1, 7, 1000, 0xFFFFFFFF):
            ks = openssl_block(kb, counter)
            cases.append({"key_name": name, "key_words": key, "counter": counter,
                          "keystream_hex": ks.hex()})
    out = {"source": "openssl enc -chacha20 (OpenSSL 3.0.2), 64 zero bytes per block",
           "rounds": 20, "cases": cases}
    path = os.path.join(ROOT, "tests", "golden", "chacha20_kat.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(cases)} cases to {path}")


if __name__ == "__main__":
    main()
