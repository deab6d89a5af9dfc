"""Device copies of the drop-in solvers' return values.

The reference drone solver returns its (x, v) as torch tensors on its device
(``drone_mppi.py:169-176``; the node calls ``xdes.to('cpu').tolist()``, ``drone.py:240``).
The engine's outputs land in host memory, so each call needs one host-to-device copy.
``OutputRing`` makes it ONE non-blocking copy of all the outputs into a fresh device
tensor per call, from a ring of pinned staging rows: a row is reused only after its copy
has run (its event; by then a whole control step has passed, so the wait is a no-op).
Two synchronous ``torch.tensor(..., device=cuda)`` copies per call used to sit on the
control step's latency path.
"""
from __future__ import annotations

import numpy as np
import torch


class OutputRing:
    def __init__(self, device: torch.device, width: int, depth: int = 8):
        self.device, self.width = device, width
        self._host = None
        self._events = None
        self._used = [False] * depth
        self._depth = depth
        self._i = 0

    def to_device(self, row: np.ndarray) -> torch.Tensor:
        """A fresh float32 tensor on ``device`` holding ``row`` (stream-ordered on the
        current stream; CPU devices get a host tensor)."""
        if self.device.type != "cuda":
            return torch.tensor(np.asarray(row, np.float32))
        if self._host is None:
            self._host = torch.zeros((self._depth, self.width), dtype=torch.float32).pin_memory()
            self._events = [torch.cuda.Event() for _ in range(self._depth)]
        i = self._i
        self._i = (i + 1) % self._depth
        if self._used[i]:
            self._events[i].synchronize()
        self._host[i].numpy()[:] = row
        t = torch.empty(self.width, dtype=torch.float32, device=self.device)
        t.copy_(self._host[i], non_blocking=True)
        self._events[i].record()
        self._used[i] = True
        return t


class LazyU:
    """The reference's ``u`` attribute (``self.u = u[0].clone()``, mppi.py:155 /
    drone_mppi.py:163): a torch tensor, built on its first read after each call from the
    call's own u0 row (``_set_u0``), so a controller that never reads it does not pay a
    ``torch.from_numpy`` (~1 us) per control call.  Assigning ``u`` stores the tensor."""

    _u_t = None
    _u_np = None

    @property
    def u(self):
        t = self._u_t
        if t is None:
            t = self._u_t = torch.from_numpy(self._u_np)
        return t

    @u.setter
    def u(self, value):
        self._u_t = value
        self._u_np = None

    def _set_u0(self, row: np.ndarray) -> None:
        """row: this call's u0 (a fresh array the engine returned, owned from here on)."""
        self._u_np = row
        self._u_t = None
