"""Worker streams for concurrent independent work inside one process (objects of a rank, frames of a filter stream).

HIP maps every stream onto one of GPU_MAX_HW_QUEUES hardware queues (4 by default) in creation order, and
torch.cuda.Stream() hands out the next stream of torch's pool.  Streams created ad hoc by successive phases of a
program therefore land on queues that depend on how many streams were created before: two "concurrent" streams can
share one hardware queue and run serially (measured: the configs[3] objects leg 19 -> 24 ms, the configs[2] stream
0.16 -> 0.20 ms/frame, depending on which leg created its streams first).  worker_streams(n) returns the same n
streams every time (created once, consecutively, per device), so concurrent workers always sit on distinct queues.
"""
from __future__ import annotations

import threading

_lock = threading.Lock()
_streams: dict = {}


def worker_streams(n: int) -> list:
    import torch

    dev = torch.cuda.current_device()
    with _lock:
        lst = _streams.setdefault(dev, [])
        while len(lst) < n:
            lst.append(torch.cuda.Stream(device=dev))
        return lst[:n]


_side: dict = {}


def side_stream(of=None):
    """A second stream paired with the current one (created once per stream): independent work of the same caller
    -- a fresh mesh's vertex normals beside its sampling's area chains -- runs there, joined by an event.  It takes the
    least stream priority the device offers, so the caller's critical-path kernels (the chains' wide passes) are
    dispatched first and the side work fills the gaps of the chains' single-wave walks."""
    import torch

    cur = of if of is not None else torch.cuda.current_stream()  # of: pair with this stream instead of the current one
    key = (cur.device_index, cur.cuda_stream)
    with _lock:
        st = _side.get(key)
        if st is None:
            least, _greatest = torch.cuda.Stream.priority_range()
            st = _side[key] = torch.cuda.Stream(device=cur.device_index, priority=least)
        return st
