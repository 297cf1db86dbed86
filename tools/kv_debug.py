"""Ad-hoc device check of the kvstore apply on a test batch (prints results + stats)."""
import os
import random
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import torch  # noqa: F401,E402
import kvstore_ref as R  # noqa: E402
from test_kv import random_blobs  # noqa: E402
from rabia_amd.kvstore import DeviceKVStore, KVStoreConfig  # noqa: E402

n, ks = int(sys.argv[1]), int(sys.argv[2])
rng = random.Random(n * 131 + ks)
blobs = random_blobs(rng, n, ks)
with DeviceKVStore(KVStoreConfig(max_value_size=64)) as dev:
    got = [int(x) for x in dev.apply_commands(blobs)]
    ref = R.KVStoreRef(max_value_size=64)
    exp = ref.apply_commands(blobs)
    for i, (g, e) in enumerate(zip(got, exp)):
        print(i, g, e, "" if g == e else "<<<", R.decode_op(blobs[i]) or blobs[i][:20])
    print(dev.stats())
    st = dev.get_state()
    print("state equal:", st == ref.state(), len(st["data"]), len(ref.state()["data"]))
