"""The bench's synthetic stripes (tools/synth.py): splitmix64
keyed by (config, global stripe index), edge stripes at global 0..2. The GPU
generator (wrapping int64 torch arithmetic) must equal the uint64 numpy twin
byte for byte, so any stripe of any N-GPU run can be regenerated on the CPU."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import synth  # noqa: E402


def test_splitmix64_known_answers():
    # splitmix64 seeded with 0: the first outputs of the published generator
    z = synth.mix64_numpy(np.arange(1, 4, dtype=np.uint64) * np.uint64(synth.GAMMA))
    assert [int(x) for x in z] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]


def test_edge_stripes_and_global_keying():
    k, L = 4, 1024
    assert (synth.stripe_numpy(3, 0, k, L) == 0).all()
    assert (synth.stripe_numpy(3, 1, k, L) == 0xFF).all()
    assert (synth.stripe_numpy(3, 2, k, L)[1] == np.arange(L) % 256).all()
    a, b = synth.stripe_numpy(3, 7, k, L), synth.stripe_numpy(5, 7, k, L)
    assert not np.array_equal(a, b) and not np.array_equal(a, synth.stripe_numpy(3, 8, k, L))


def test_torch_generator_matches_numpy_cpu():
    k, p, L = 10, 4, 4096
    st = torch.zeros((6, k + p, L), dtype=torch.uint8)
    synth.fill_data_rows(torch, st, 3, 1, k, p, batch=4)  # global stripes 1..6: two edges + randoms
    for i in range(6):
        assert np.array_equal(st[i, p:].numpy(), synth.stripe_numpy(3, 1 + i, k, L)), i
    assert (st[:, :p] == 0).all()


@pytest.mark.gpu
def test_torch_generator_matches_numpy_gpu(cuda):
    k, p, L = 12, 4, 256 << 10
    st = torch.zeros((5, k + p, L), dtype=torch.uint8, device="cuda")
    synth.fill_data_rows(torch, st, 5, 1021, k, p)
    host = st.cpu().numpy()
    for i in range(5):
        assert np.array_equal(host[i, p:], synth.stripe_numpy(5, 1021 + i, k, L)), i
