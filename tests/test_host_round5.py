"""Round-5 host-side tests (no GPU): cirtorch.utils.image.normalize against the
reference formula, and the ASan build of librr's host half."""

import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "image-retrieval-for-image-based-localization_amd", "csrc")


def _reference_normalize(data, mean, std):
    """the arithmetic of cirtorch/utils/image.py:86-127 (4-D batches)"""
    shape = data.shape
    mean = torch.as_tensor(mean, dtype=data.dtype)
    std = torch.as_tensor(std, dtype=data.dtype)
    if mean.shape:
        mean = mean[..., :, None]
    if std.shape:
        std = std[..., :, None]
    return ((data.view(shape[0], shape[1], -1) - mean) / std).view(shape)


@pytest.mark.parametrize("stats", ["channel", "batch", "scalar", "list"])
def test_normalize_bit_identical_to_reference(stats):
    from cirtorch.utils.image import normalize
    g = torch.Generator().manual_seed(3)
    x = torch.rand((3, 3, 17, 29), generator=g)
    if stats == "channel":
        m, s = torch.tensor([0.485, 0.456, 0.406]), torch.tensor([0.229, 0.224, 0.225])
    elif stats == "batch":
        m, s = torch.rand((3, 3), generator=g), torch.rand((3, 3), generator=g) + 0.5
    elif stats == "scalar":
        m, s = torch.tensor(0.5), torch.tensor(0.25)
    else:
        m, s = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    got = normalize(x, m, s)
    assert torch.equal(got, _reference_normalize(x, m, s))
    assert torch.equal(x, torch.rand((3, 3, 17, 29), generator=torch.Generator().manual_seed(3)))  # input untouched


def test_normalize_errors():
    from cirtorch.utils.image import normalize
    x = torch.rand((2, 3, 4, 4))
    with pytest.raises(ValueError):
        normalize(x, [0.1, 0.2], [1.0, 1.0, 1.0])
    with pytest.raises(TypeError):
        normalize(x.numpy(), [0.1, 0.2, 0.3], [1.0, 1.0, 1.0])
    with pytest.raises(TypeError):
        normalize(x, "mean", [1.0, 1.0, 1.0])
    # [N, C] statistics index dims -4 / -3: a 5-D [B, N, C, H, W] batch takes [N, C] stats,
    # a stat shaped like the leading (B, N) dims is refused
    x5 = torch.rand((2, 4, 3, 5, 5))
    m5 = torch.rand((4, 3))
    got = normalize(x5, m5, torch.ones(4, 3))
    assert torch.equal(got, x5 - m5[:, :, None, None])
    with pytest.raises(ValueError):
        normalize(x5, torch.rand((2, 4)), torch.ones(2, 4))
    with pytest.raises(ValueError):
        normalize(torch.rand((3, 5, 5)), torch.rand((1, 3)), torch.ones(1, 3))


def test_host_half_under_asan():
    """`make asan`: librr's host half (every source but the GEMM kernels' TU) built
    with -fsanitize=address, driven by tests/asan/asan_driver.cpp on this GPU-less
    host -- workspace sizing, argument checks, ragged-table packing of 150 images,
    tuning keys, the RCCL id -- with no AddressSanitizer report."""
    if shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no hipcc / make")
    # the regular build provides rr_gemm.o (a no-op when librr.so is current)
    subprocess.run(["make", "-C", CSRC, "-j8"], check=True, capture_output=True, timeout=1800)
    subprocess.run(["make", "-C", CSRC, "-j8", "asan"], check=True, capture_output=True, timeout=1800)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=86", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([os.path.join(CSRC, "build_asan", "asan_driver")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert r.stdout.strip().endswith("ASAN-DRIVER OK")


def test_proc_decoder_close_after_worker_death():
    """on an error path (a decode worker died with copies pending),
    ProcDecoder.close() waits for every pending copy's event before unpinning the
    ring, and unlinks the shared-memory segment even though a view into it is
    still alive (shm.close() raises BufferError then)."""
    from cirtorch.utils import decode_procs as dp
    d = dp.ProcDecoder(2, 4, slot_bytes=64 << 10)
    name = d.shm.name
    assert os.path.exists("/dev/shm/" + name)

    class _Ev:
        waited = 0

        def synchronize(self):
            _Ev.waited += 1

        def query(self):
            return False

    d.busy = [(_Ev(), [0]), (_Ev(), [1, 2])]
    view = np.frombuffer(d.shm.buf, np.uint8)[:16]     # a live export of the ring
    d._procs[0].kill()
    d._procs[0].join(10)
    assert d.worker_died()
    d.close()
    assert _Ev.waited == 2 and d.busy == []
    assert not os.path.exists("/dev/shm/" + name)
    del view
