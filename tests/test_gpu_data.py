"""f4: the training data path on the device (u3d.data, data.hip) against the numpy / scipy restatement of
MOTSDataset.py (oracle/ref_cpu.py: truncate, pad, crop, transpose; batchgenerators' blur and contrast). The crop
offsets are drawn with the same seeded numpy RandomState on both sides (the reference's np.random calls); the
batchgenerators draw sequence itself is unpinned (library absent), each applied operation is pinned here."""
import numpy as np
import pytest
import torch

from oracle import ref_cpu as O

pytestmark = pytest.mark.gpu


def _case(shape, seed):
    rng = np.random.default_rng(seed)
    image = rng.integers(-1200, 1500, size=shape).astype(np.float32)
    label = rng.integers(0, 14, size=shape).astype(np.float32)
    catlas = rng.uniform(0, 1, size=(13,) + shape).astype(np.float32)
    return image, label, catlas


@pytest.mark.parametrize("name,shape", [("0007", (20, 30, 12)), ("0555", (20, 30, 12)), ("0031", (40, 44, 30)),
                                        ("0612", (40, 44, 30))])
def test_crop_patch_vs_reference_restatement(gpu, name, shape):
    from u3d import data
    image, label, catlas = _case(shape, 3)
    crop = (8, 12, 16)  # (crop_d, crop_h, crop_w) as the dataset stores them
    ri, rl, rc = O.get_item_tensors(image, label, catlas, name, crop, np.random.RandomState(5))
    gi, gl, gc = data.crop_patch(torch.from_numpy(image).to(gpu), torch.from_numpy(label).to(gpu),
                                 torch.from_numpy(catlas).to(gpu), name, crop, rng=np.random.RandomState(5))
    assert gi.shape == ri.shape and gl.shape == rl.shape and gc.shape == rc.shape
    np.testing.assert_allclose(gi.cpu().numpy(), ri, rtol=1e-5, atol=1e-5)
    assert np.array_equal(gl.cpu().numpy(), rl)
    np.testing.assert_allclose(gc.cpu().numpy(), rc.astype(np.float32), rtol=0, atol=0)


@pytest.mark.parametrize("tag", ["ct_small", "ct_big", "mri_small", "mri_big", "ct_valid", "mri_valid"])
def test_crop_patch_vs_reference_fixture(gpu, tag):
    """f4 pinned on the reference's own lines (G15: MOTSDataset.py:171-186, :269-297, :370-397 exec'd in
    tests/golden/gen_golden.py::g15 on CT int16 / MRI float32 volumes, train and valid): crop offsets drawn from the
    same seeded RandomState in the reference's order (checked against the recorded draws), labels and atlas crops
    bit-exact, the normalised image within 1e-6 (CT: one fp32 division vs numpy's float64 division then cast; MRI:
    fp64 device statistics vs numpy's float32 pairwise mean / std)."""
    from conftest import golden
    from u3d import data
    g = golden("g15_crop_patch.npz")
    crop = tuple(int(v) for v in g[f"{tag}_crop"])
    rs = np.random.RandomState(int(g[f"{tag}_seed"]))
    draws = []

    class Rec:
        def randint(self, *a):
            draws.append(int(rs.randint(*a)))
            return draws[-1]
    f = lambda k: torch.from_numpy(g[f"{tag}_{k}"].astype(np.float32)).to(gpu)  # noqa: E731 - host cast (exact)
    gi, gl, gc = data.crop_patch(f("image_in"), f("label_in"), f("catlas_in"), str(g[f"{tag}_name"]), crop,
                                 usage=str(g[f"{tag}_usage"]), rng=Rec())
    assert draws == g[f"{tag}_draws"].tolist()
    ri, rl, rc = g[f"{tag}_image"], g[f"{tag}_label"], g[f"{tag}_catlas"]
    assert gi.shape == ri.shape and gl.shape == rl.shape and gc.shape == rc.shape
    assert np.array_equal(gl.cpu().numpy(), rl)
    assert np.array_equal(gc.cpu().numpy(), rc)
    np.testing.assert_allclose(gi.cpu().numpy(), ri, rtol=0, atol=1e-6)


@pytest.mark.parametrize("sigma,shape", [(0.5, (9, 10, 11)), (0.83, (16, 12, 20)), (1.0, (3, 17, 5))])
def test_blur_vs_scipy(gpu, sigma, shape):
    from u3d import data
    x = np.random.default_rng(1).standard_normal(shape).astype(np.float32)
    y = data.gaussian_blur(torch.from_numpy(x).to(gpu), sigma)
    np.testing.assert_allclose(y.cpu().numpy(), O.aug_blur(x, sigma), rtol=1e-5, atol=1e-6)


def test_contrast_affine_stats(gpu):
    from u3d import data
    from u3d._lib import call
    from u3d import ops
    x = np.random.default_rng(2).standard_normal((7, 9, 11)).astype(np.float32) * 3 + 1
    t = torch.from_numpy(x).to(gpu)
    st = data.volume_stats(t).cpu().numpy()
    np.testing.assert_allclose(st, [x.mean(), x.std(), x.min(), x.max()], rtol=1e-5, atol=1e-6)
    stp = data.volume_stats(t, count=x.size + 500).cpu().numpy()
    xp = np.concatenate([x.reshape(-1), np.zeros(500, np.float32)])
    np.testing.assert_allclose(stp, [xp.mean(), xp.std(), xp.min(), xp.max()], rtol=1e-5, atol=1e-6)
    for f in (0.8, 1.2):
        u = t.clone()
        call("u3d_aug_contrast", u.data_ptr(), u.numel(), f, data.volume_stats(u).data_ptr(), 1, ops._stream())
        np.testing.assert_allclose(u.cpu().numpy(), O.aug_contrast(x, f), rtol=1e-5, atol=1e-5)
    u = t.clone()
    call("u3d_aug_affine", u.data_ptr(), u.numel(), 1.1, -0.05, ops._stream())
    np.testing.assert_allclose(u.cpu().numpy(), x * 1.1 - 0.05, rtol=1e-6, atol=1e-6)


def test_noise_statistics_and_determinism(gpu):
    from u3d._lib import call
    from u3d import ops
    z = torch.zeros(1 << 20, device=gpu)
    call("u3d_aug_noise", z.data_ptr(), z.numel(), 0.07, 1234, ops._stream())
    z2 = torch.zeros_like(z)
    call("u3d_aug_noise", z2.data_ptr(), z2.numel(), 0.07, 1234, ops._stream())
    assert torch.equal(z, z2)
    assert abs(z.mean().item()) < 1e-3 and abs(z.std().item() / 0.07 - 1) < 1e-2
    assert abs(((z / 0.07) ** 4).mean().item() - 3) < 0.05   # Gaussian kurtosis


def test_train_transform_replays_on_the_restatement(gpu):
    """Every operation train_transform applied (its log) replayed in order on the numpy/scipy restatement gives the
    same batch (seeds chosen so that blur, brightness and contrast fire; noise checked separately above)."""
    from u3d import data
    x = np.random.default_rng(4).standard_normal((3, 1, 6, 8, 10)).astype(np.float32)
    fired = set()
    for seed in range(40):
        out, log = data.train_transform(torch.from_numpy(x).to(gpu), rng=np.random.RandomState(seed))
        if any(op[0] == "noise" for op in log):
            continue
        ref = x.copy()
        for op in log:
            fired.add(op[0])
            b, c = op[1], op[2]
            if op[0] == "blur":
                ref[b, c] = O.aug_blur(ref[b, c], op[3])
            elif op[0] == "mul":
                ref[b, c] = ref[b, c] * np.float32(op[3])
            elif op[0] == "add":
                ref[b, c] = ref[b, c] * np.float32(1.0) + np.float32(op[3])
            elif op[0] == "contrast":
                ref[b, c] = O.aug_contrast(ref[b, c], op[3])
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    assert {"blur", "mul", "add", "contrast"} <= fired
