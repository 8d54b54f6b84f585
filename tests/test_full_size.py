"""Every BASELINE config at its full bench size and layout (bench.py CONFIGS, the
recommended row pitch), checked through properties that do not need the CPU oracle to
re-encode gigabytes:

* round trip: encode, erase the config's lost shards (or, for the encode-only configs, data
  shard 0 and a parity shard), reconstruct, compare every byte with the encoded original;
* linearity: encode(X xor Y) == encode(X) xor encode(Y), over every block;
* a sample of blocks re-encoded by the oracle (test-only), byte for byte.
"""
import numpy as np
import pytest

import oracle_lib as orc

torch = pytest.importorskip("torch")
rsmi = pytest.importorskip("rsmi")

pytestmark = pytest.mark.gpu

# (k, m, block KiB, blocks, lost shards, data_only) -- bench.py CONFIGS
CONFIGS = {
    "rs10_4_256k": (10, 4, 256, 4096, [0], True),
    "rs4_2_256k": (4, 2, 256, 4096, [0, 5], False),
    "rs10_4_1m": (10, 4, 1024, 1024, [3, 12], False),
    "rs16_4_4m": (16, 4, 4096, 256, [0, 9], True),
    "rs2_1_256k": (2, 1, 256, 4096, [1], True),
}


def _blocks(k, n, S, p, nb, B, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    x = torch.randint(0, 256, (nb, n, p), dtype=torch.uint8, device="cuda", generator=g)
    x[:, :, S:] = 0
    if k * S > B:  # Split's zero padding of the last data row
        x[:, k - 1, S - (k * S - B):S] = 0
    return x


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_full_size_properties(name):
    k, m, kib, nb, lost, data_only = CONFIGS[name]
    n, B = k + m, kib * 1024
    S = (B + k - 1) // k
    p = rsmi.recommended_pitch(S)
    sh = torch.cuda.current_stream().cuda_stream
    x = _blocks(k, n, S, p, nb, B, 7)
    y = _blocks(k, n, S, p, nb, B, 8)
    with rsmi.Codec(k, m) as c:
        enc = lambda t: c.encode_batch_dev(t.data_ptr(), p, n * p, t.data_ptr() + k * p, p, n * p, S, nb, sh)
        enc(x)
        enc(y)
        z = x ^ y  # data rows xor; parity rows recomputed below
        z[:, k:, :] = 0
        enc(z)
        torch.cuda.synchronize()
        assert torch.equal(z[:, k:, :S], x[:, k:, :S] ^ y[:, k:, :S]), "encode is not linear"
        orig = x.clone()
        x[:, lost, :] = 0
        present = [i not in lost for i in range(n)]
        c.reconstruct_batch_dev(x.data_ptr(), p, n * p, S, nb, present, data_only, sh)
        torch.cuda.synchronize()
    rebuilt = [i for i in lost if i < k or not data_only]
    assert torch.equal(x[:, rebuilt, :S], orig[:, rebuilt, :S]), "round trip differs"
    kept = [i for i in lost if i not in rebuilt]
    assert not x[:, kept, :].any(), "a row the call did not ask for was written"
    others = [i for i in range(n) if i not in lost]
    assert torch.equal(x[:, others, :], orig[:, others, :]), "a present row was touched"
    idx = sorted({0, 1, nb // 2, nb - 1})
    host = orig[idx].cpu().numpy()
    want = orc.encode_fast(k, m, np.ascontiguousarray(host[:, :k, :S]))
    assert np.array_equal(host[:, k:, :S], want)
