"""CPU: seeded synthetic inputs are deterministic and sharding-invariant (global-index seeding)."""
import numpy as np

from admm_deconv import parallel, synth


def test_psf_normalised():
    for k, s in ((9, 1.2), (15, 2.5)):
        p = synth.gaussian_psf(k, s)
        assert p.shape == (k, k) and abs(p.sum() - 1) < 1e-6 and np.allclose(p, p.T)
    assert abs(synth.box_psf_row(7).sum() - 1) < 1e-6


def test_batch_deterministic_and_shard_invariant():
    psf = synth.gaussian_psf(5, 1.0)
    a = synth.make_batch(6, 32, 32, psf)
    b = synth.make_batch(6, 32, 32, psf)
    assert np.array_equal(a, b)
    parts = [synth.make_batch(c, 32, 32, psf, g0=s) for s, c in (parallel.shard_range(6, 4, r) for r in range(4))]
    assert np.array_equal(np.concatenate(parts), a)


def test_shard_range_covers():
    for total in (0, 1, 7, 512, 2048):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = parallel.shard_range(total, world, r)
                seen.extend(range(s, s + c))
            assert seen == list(range(total))
