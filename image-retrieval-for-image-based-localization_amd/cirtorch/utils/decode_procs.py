"""Image-file decoding in worker processes for ``extract_vectors``
(``scripts/test.py:236-238`` -> ``cirtorch/datasets/genericdataset.py``'s PIL
loader: open, RGB, bbx crop, ``thumbnail`` to ``imsize``).

PIL's JPEG / PNG decoders release the GIL, but the Python around them (the
chunked load loop, ``convert``, the array export) does not: decode threads
stop scaling at ~1.6k 1024x768 JPEGs/s on 16 host threads.  Here W spawned
worker processes (numpy + PIL only, no GPU) decode each file straight into a
slot of one shared-memory ring, which the parent page-locks once
(``hipHostRegister`` through ``torch.cuda.cudart()``): a decoded image is a
pinned [H, W, 3] uint8 view that the chain's H2D copy reads directly, and the
slot goes back to the free list when that copy's event has completed.  Images
larger than a slot come back pickled (plain host memory).

Host-side plumbing only: the pixels are the same bytes the thread path
produces (``GF_net._load_pil``), so descriptors are identical.
"""

import os
import threading

import numpy as np


class DecoderFailure(RuntimeError):
    """the process decoder itself failed (a worker died, e.g. SIGBUS on a full
    /dev/shm): extract_vectors falls back to its decode threads"""

_SHM = None  # worker side: the parent's ring


def _worker_init(name):
    global _SHM
    from multiprocessing import shared_memory
    # (spawned workers share the parent's resource tracker, so attaching registers
    # nothing new; the parent unlinks the segment)
    _SHM = shared_memory.SharedMemory(name=name)


def _load(path, imsize, bbx):
    """GF_net._load_pil, restated for a process that does not import torch (an RGB
    file skips convert("RGB"), which would only copy it: same pixels)"""
    from PIL import Image
    with open(path, "rb") as f:
        img = Image.open(f)
        img.load()
    if img.mode != "RGB":
        img = img.convert("RGB")
    if bbx is not None:
        img = img.crop(bbx)
    if imsize is not None:
        img.thumbnail((imsize, imsize), Image.LANCZOS)
    return img


def _decode_into(args):
    path, imsize, bbx, off, cap = args
    img = _load(path, imsize, bbx)
    data = img.tobytes()  # raw RGB rows: one copy, then one into the ring
    shape = (img.height, img.width, 3)
    if len(data) > cap:
        return shape, np.frombuffer(data, np.uint8).reshape(shape).copy()
    _SHM.buf[off:off + len(data)] = data
    return shape, None


def _decode_group(group):
    """several files per task: one IPC round trip (pickling in the parent holds
    its GIL) per group instead of per image"""
    return [_decode_into(g) for g in group]


class _Pending:
    def __init__(self, owner, slot, res, k=None):
        self.owner, self.slot, self.res, self.k = owner, slot, res, k

    def result(self):
        import torch
        # wait in slices: a worker that died (its task is lost for good) is noticed
        # within a second instead of at the timeout
        for _ in range(300):
            if self.res.ready():
                break
            self.res.wait(1.0)
            if not self.res.ready() and self.owner.worker_died():
                raise DecoderFailure("a decode worker process died")
        out = self.res.get(timeout=1.0)
        shape, big = out if self.k is None else out[self.k]
        if big is not None:
            self.owner._give_back([self.slot])
            return torch.from_numpy(big)
        t = torch.from_numpy(np.ndarray(shape, np.uint8, buffer=self.owner.shm.buf,
                                        offset=self.slot * self.owner.slot_bytes))
        with self.owner.lock:
            self.owner.slot_of[t.data_ptr()] = self.slot
        return t


class ProcDecoder:
    """W decode processes + a page-locked shared-memory ring of `nslots` slots."""

    def __init__(self, workers, nslots, slot_bytes=1024 * 1024 * 3):
        import multiprocessing as mp
        from multiprocessing import shared_memory
        import torch
        self.slot_bytes, self.nslots, self.workers = slot_bytes, nslots, workers
        self.shm = shared_memory.SharedMemory(create=True, size=nslots * slot_bytes)
        buf = np.frombuffer(self.shm.buf, np.uint8)
        self.registered = False
        try:
            rc = torch.cuda.cudart().cudaHostRegister(buf.ctypes.data, buf.nbytes, 0)
            self.registered = int(rc) == 0
        except Exception:
            self.registered = False
        self._base = buf.ctypes.data
        del buf
        # Spawned workers would re-run the parent's __main__ script (bench.py, a test
        # runner, stdin): they import only this module, so the pool is started while
        # __main__ is a bare module with no file to re-run.
        import sys
        import types
        main = sys.modules["__main__"]
        sys.modules["__main__"] = types.ModuleType("__main__")
        try:
            self.pool = mp.get_context("spawn").Pool(workers, initializer=_worker_init, initargs=(self.shm.name,))
        finally:
            sys.modules["__main__"] = main
        self._procs = list(getattr(self.pool, "_pool", []))  # the workers as started
        # each worker's sentinel: a pipe end that becomes readable when the process ends,
        # whoever reaps it (the Pool's maintenance thread polls exitcode concurrently, and a
        # racing Popen.poll() can miss the exit: ECHILD -> None)
        self._sentinels = [p.sentinel for p in self._procs]
        self._died = False
        self.lock = threading.Lock()
        self.free = list(range(nslots))
        self.busy = []      # (event, [slots]) waiting for their H2D copy
        self.slot_of = {}   # data_ptr of a handed-out view -> slot

    def worker_died(self):
        """True once any of the started workers has exited (multiprocessing.Pool
        replaces a dead worker but never re-runs the task it held)"""
        if not self._died and self._sentinels:
            from multiprocessing.connection import wait
            try:
                self._died = bool(wait(self._sentinels, timeout=0))
            except (OSError, ValueError):    # a sentinel already closed: its process is gone
                self._died = True
        return self._died

    def _reclaim(self, block):
        keep = []
        for ev, slots in self.busy:
            if ev.query():
                self.free.extend(slots)
            else:
                keep.append((ev, slots))
        self.busy = keep
        if block and not self.free and self.busy:
            ev, slots = self.busy.pop(0)
            ev.synchronize()
            self.free.extend(slots)

    def _give_back(self, slots):
        with self.lock:
            self.free.extend(slots)

    def submit(self, path, imsize, bbx):
        with self.lock:
            self._reclaim(block=False)
            if not self.free:
                self._reclaim(block=True)
            if not self.free:
                raise RuntimeError("ProcDecoder: every slot is held by an undelivered image (ring too small)")
            slot = self.free.pop()
        res = self.pool.apply_async(_decode_into, ((path, imsize, bbx, slot * self.slot_bytes, self.slot_bytes),))
        return _Pending(self, slot, res)

    def submit_group(self, items):
        """items: [(path, imsize, bbx)] -> one pending image each, decoded by one task"""
        slots = []
        with self.lock:
            for _ in items:
                self._reclaim(block=False)
                if not self.free:
                    self._reclaim(block=True)
                if not self.free:
                    self.free.extend(slots)
                    raise RuntimeError("ProcDecoder: every slot is held by an undelivered image (ring too small)")
                slots.append(self.free.pop())
        res = self.pool.apply_async(_decode_group, ([(p, s_, b, sl * self.slot_bytes, self.slot_bytes)
                                                     for (p, s_, b), sl in zip(items, slots)],))
        return [_Pending(self, sl, res, k) for k, sl in enumerate(slots)]

    def owns(self, t):
        return t.data_ptr() in self.slot_of

    def release(self, views, event):
        """views: tensors from result(); event: recorded after the copies that read them"""
        with self.lock:
            slots = [self.slot_of.pop(v.data_ptr()) for v in views if v.data_ptr() in self.slot_of]
            if slots:
                self.busy.append((event, slots))

    def close(self):
        """terminate the workers, then -- only once no H2D copy can still read the
        ring -- unpin and release it.  Safe on an error path: copies listed in
        `busy` are waited for, and so is every other queued copy (a view handed out
        but never released may have one in flight), before cudaHostUnregister;
        the segment is unlinked even when unmapping fails because views into it are
        still alive (BufferError), so /dev/shm is returned when they die."""
        import torch
        try:
            self.pool.terminate()
        except Exception:
            pass
        with self.lock:
            busy, self.busy = self.busy, []
        for ev, _ in busy:
            try:
                ev.synchronize()
            except Exception:
                pass
        if self.registered:
            try:
                if torch.cuda.is_initialized():
                    torch.cuda.synchronize()
            except Exception:
                pass
            try:
                torch.cuda.cudart().cudaHostUnregister(self._base)
            except Exception:
                pass
            self.registered = False
        try:
            self.shm.close()
        except Exception:   # BufferError: views into the ring are still alive
            pass
        try:
            self.shm.unlink()
        except Exception:   # already unlinked
            pass


_DEC = {}

RING_MAX_BYTES = 2 << 30   # never more than 2 GiB of /dev/shm
SHM_SHARE = 0.5            # nor more than half of what /dev/shm has free


def slot_bytes_for(image_size):
    """ring slot size: one decoded RGB image of at most image_size x image_size
    (thumbnail), or a 1024 x 1024 one when the size is not capped; larger images
    come back pickled instead"""
    side = int(image_size) if image_size else 1024
    return max(64 << 10, (side * side * 3 + 4095) // 4096 * 4096)


def shm_free_bytes(path="/dev/shm"):
    try:
        st = os.statvfs(path)
        return st.f_bavail * st.f_frsize
    except OSError:
        return 0


def drop():
    """close and forget the cached decoder (after an error: its slots may be held
    by deliveries that will never happen)"""
    d = _DEC.pop("d", None)
    if d is not None:
        d.close()


def get(workers, nslots, slot_bytes=3 << 20):
    """the process decoder of this host process (created on first use, kept: the
    workers' start-up is paid once); re-created if asked for more workers / slots /
    larger slots.  None when the ring does not fit (RING_MAX_BYTES, or SHM_SHARE of
    the free /dev/shm: a worker writing past a full tmpfs dies of SIGBUS) or cannot
    be page-locked: the caller decodes on threads instead."""
    import atexit
    d = _DEC.get("d")
    if d is not None and d.workers >= workers and d.nslots >= nslots and d.slot_bytes >= slot_bytes:
        return d
    drop()
    need = nslots * slot_bytes
    if need > RING_MAX_BYTES or need > SHM_SHARE * shm_free_bytes():
        return None
    try:
        d = ProcDecoder(workers, nslots, slot_bytes)
    except (OSError, ValueError, RuntimeError):
        return None
    if not d.registered:
        d.close()
        return None
    _DEC["d"] = d
    if not _DEC.get("atexit"):
        atexit.register(lambda: _DEC["d"].close() if _DEC.get("d") else None)
        _DEC["atexit"] = True
    return d
