"""Stream ordering for the C-ABI launches (include/mhe.h: every call only enqueues
work on the stream it is given).

A launch on a stream ``s`` other than torch's current stream needs three things the
C-ABI cannot do for the caller:
  * ``s`` must wait for the current stream, where the inputs were produced or
    staged (and for the event that marks the device constants as built);
  * tensors the launch reads or writes must not return to torch's caching
    allocator (and be handed to another stream) before ``s`` is done with them:
    ``record_stream(s)``;
  * temporaries and outputs are allocated under ``torch.cuda.stream(s)`` so their
    reuse is ordered on ``s``.
The caller consumes outputs on ``s`` or makes its own stream wait for ``s``, as with
any torch side stream.
"""
import contextlib

import torch


@contextlib.contextmanager
def launch_stream(stream, device, wait_events=()):
    """Yields (s, cur): the torch stream to launch on (``stream`` or the current one)
    and the caller's current stream; inside the block ``s`` is torch's current
    stream, so staging copies and allocations are ordered on it."""
    cur = torch.cuda.current_stream(device)
    s = cur if stream is None else stream
    if s != cur:
        s.wait_stream(cur)
    for e in wait_events:
        if e is not None:
            s.wait_event(e)
    with torch.cuda.stream(s):
        yield s, cur


def keep_alive(s, cur, *tensors):
    """record_stream(s) on every tensor a launch on ``s`` touches (no-op when ``s``
    is the caller's current stream ``cur``, where allocator reuse is already ordered)."""
    if s == cur:
        return
    for t in tensors:
        if isinstance(t, torch.Tensor):
            t.record_stream(s)
