"""Replays tests/test_kv.py::test_gpu_random_batches_vs_oracle's smallest cases
batch by batch, printing commands, device vs restatement results, the device's
stats and raw table after every batch (for finding where a keyed-path change goes
wrong). Run on the GPU box."""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import kvstore_ref as R  # noqa: E402
from test_kv import random_blobs  # noqa: E402
from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig  # noqa: E402

for n, key_space, batches in ((1, 1, 3), (37, 5, 4)):
    rng = random.Random(n * 131 + key_space)
    dev = DeviceKVStore(KVStoreConfig(max_value_size=64))
    ref = R.KVStoreRef(max_value_size=64)
    for b in range(batches):
        blobs = random_blobs(rng, n, key_space)
        got = [int(x) for x in dev.apply_commands(blobs)]
        exp = ref.apply_commands(blobs)
        print(f"n={n} batch {b}: kinds={[x[0] for x in blobs][:12]} got={got[:12]} exp={exp[:12]} same={got == exp}")
        print("   stats", dev.stats())
        st = dev.get_state()
        if n == 1:
            import ctypes
            from rabia_amd import _native as NN
            slots = ctypes.c_uint64()
            NN.check_kv(dev.lib.rg_kv_table_slots(dev.kv, ctypes.byref(slots)), dev.kv)
            hs = np.zeros(int(slots.value), np.uint64)
            en = np.zeros((int(slots.value), 4), np.uint64)
            hp = np.zeros(4096, np.uint8)
            NN.check_kv(dev.lib.rg_kv_dump(dev.kv, hs.ctypes.data, en.ctypes.data, hp.ctypes.data, hp.size), dev.kv)
            for q in np.nonzero(hs)[0]:
                print("   slot", int(q), hex(int(hs[q])), [hex(int(x)) for x in en[q]])
        print("   dev data", sorted(st["data"].items())[:6])
        print("   ref data", sorted(ref.state()["data"].items())[:6] if hasattr(ref, "state") else None)
    dev.close()
