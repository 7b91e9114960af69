"""Pubsub ingest rate: K peers' gradient frames of one
partition, each Marshall_Packet'ed (MyIPFSClass.java:990-1017) and
base64url-encoded twice as they travel over IPFS pubsub (IPLS.java:855-859),
start as host text; ipls_agg_ingest_pubsub copies them to the GPU, decodes
both layers, parses the frames and folds the payloads.  Reports the rate in
gradient bytes (K*L*8 per batch) and in host text bytes (what crosses PCIe),
against the 56 GB/s PCIe ceiling.  Dev tool."""
import base64
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ipls-java-api_amd")]
import ipls  # noqa: E402


def main(L=1048576, K=32, reps=5):
    rng = np.random.default_rng(1)
    texts = []
    for k in range(K):
        g = rng.standard_normal(L) * 1e-2
        g[-1] = 1.0
        fr = ipls.frame_encode(g, 0, 7, 3, b"QmPeer%02d" % k)          # pid 3, partition 0, iteration 7
        texts.append(base64.urlsafe_b64encode(base64.urlsafe_b64encode(fr)))
    text_bytes = sum(len(t) for t in texts)
    agg = ipls.Aggregator(n_partitions=1, bucket_len=L)
    n, st = agg.ingest_pubsub(texts)                                    # warm
    assert n == K and all(s == 0 for s in st), st
    agg.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        agg.ingest_pubsub(texts)
    agg.sync()
    dt = (time.perf_counter() - t0) / reps
    print(f"ingest K={K} frames x L={L} doubles (double base64url, {text_bytes / 1e6:.0f} MB of text per batch): "
          f"{dt * 1e3:.2f} ms per batch = {K * L * 8 / dt / 1e9:.2f} GB/s of gradients, "
          f"{text_bytes / dt / 1e9:.2f} GB/s of pubsub text (PCIe ceiling ~56 GB/s)")
    agg.close()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
