"""Data path timing: crop_patch of a 512 x 512 x 160 CT / MRI volume to the 64 x 192 x 192
training patch (+ label + 13-channel atlas) and train_transform on the patch with every transform forced on.
Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "multimodal-pl_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


class _Always:
    """RandomState stand-in that fires every transform (uniform -> low end) — timing only."""

    def __init__(self):
        self.r = np.random.RandomState(0)

    def uniform(self, a=0.0, b=1.0):
        return a if (a, b) == (0.0, 1.0) else self.r.uniform(a, b)

    def normal(self, m, s):
        return self.r.normal(m, s)

    def randint(self, *a):
        return self.r.randint(*a)


def main():
    from u3d import data
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    vol = (torch.rand((512, 512, 160), generator=g) * 2500 - 1200).to(dev)
    lab = torch.randint(0, 14, (512, 512, 160), generator=g).float().to(dev)
    cat = torch.rand((13, 512, 512, 160), generator=g).to(dev)
    res = {}
    for name in ("0007", "0555"):
        for _ in range(2):
            data.crop_patch(vol, lab, cat, name, (64, 192, 192), rng=np.random.RandomState(0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            img, _, _ = data.crop_patch(vol, lab, cat, name, (64, 192, 192), rng=np.random.RandomState(0))
        torch.cuda.synchronize()
        res["crop_ms_" + ("ct" if name == "0007" else "mri")] = (time.perf_counter() - t0) * 100
    batch = img.unsqueeze(0)
    data.train_transform(batch, rng=_Always())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        _, log = data.train_transform(batch, rng=_Always())
    torch.cuda.synchronize()
    res["transform_all_ms"] = (time.perf_counter() - t0) * 100
    res["ops"] = [op[0] for op in log]
    print(json.dumps({"metric": "device data path ms per patch (64x192x192 from a 512x512x160 volume)", **res}))


if __name__ == "__main__":
    main()
