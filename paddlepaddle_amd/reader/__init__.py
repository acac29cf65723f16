"""paddle.reader: legacy reader-creator decorators (reference python/paddle/reader/decorator.py).
A *reader* is a zero-argument callable returning an iterator of samples."""
from __future__ import annotations

import itertools
import queue
import random
import threading

__all__ = []


class ComposeNotAligned(ValueError):
    pass


def cache(reader):
    """Read everything once, replay from memory afterwards."""
    all_data = tuple(reader())

    def __impl__():
        yield from all_data
    return __impl__


def map_readers(func, *readers):
    def reader():
        for e in map(func, *[r() for r in readers]):
            yield e
    return reader


def shuffle(reader, buf_size):
    def data_reader():
        buf = []
        for e in reader():
            buf.append(e)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        if buf:
            random.shuffle(buf)
            yield from buf
    return data_reader


def chain(*readers):
    def reader():
        return itertools.chain(*[r() for r in readers])
    return reader


def compose(*readers, check_alignment=True):
    def make_tuple(x):
        return x if isinstance(x, tuple) else (x,)

    def reader():
        rs = [r() for r in readers]
        if not check_alignment:
            for outputs in zip(*rs):
                yield sum(map(make_tuple, outputs), ())
        else:
            for outputs in itertools.zip_longest(*rs):
                for o in outputs:
                    if o is None:
                        raise ComposeNotAligned("outputs of readers are not aligned.")
                yield sum(map(make_tuple, outputs), ())
    return reader


def buffered(reader, size):
    """Prefetch up to ``size`` samples on a background thread."""
    end = object()

    def data_reader():
        q = queue.Queue(maxsize=size)

        def fill():
            for d in reader():
                q.put(d)
            q.put(end)
        t = threading.Thread(target=fill, daemon=True)
        t.start()
        e = q.get()
        while e is not end:
            yield e
            e = q.get()
    return data_reader


def firstn(reader, n):
    def firstn_reader():
        for i, item in enumerate(reader()):
            if i == n:
                break
            yield item
    return firstn_reader


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    """Map samples with ``process_num`` worker threads (order kept when ``order``)."""
    end = object()

    def xreader():
        in_q, out_q = queue.Queue(buffer_size), queue.Queue(buffer_size)

        def feed():
            for i, s in enumerate(reader()):
                in_q.put((i, s))
            for _ in range(process_num):
                in_q.put(end)

        def work():
            while True:
                item = in_q.get()
                if item is end:
                    out_q.put(end)
                    return
                i, s = item
                out_q.put((i, mapper(s)))
        threading.Thread(target=feed, daemon=True).start()
        for _ in range(process_num):
            threading.Thread(target=work, daemon=True).start()
        finished, nxt, pending = 0, 0, {}
        while finished < process_num:
            item = out_q.get()
            if item is end:
                finished += 1
                continue
            if not order:
                yield item[1]
                continue
            pending[item[0]] = item[1]
            while nxt in pending:
                yield pending.pop(nxt)
                nxt += 1
        while order and nxt in pending:
            yield pending.pop(nxt)
            nxt += 1
    return xreader


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    """Interleave several readers (threads here; the samples are produced by Python code either way)."""
    end = object()

    def reader():
        q = queue.Queue(queue_size)

        def run(r):
            for s in r():
                q.put(s)
            q.put(end)
        for r in readers:
            threading.Thread(target=run, args=(r,), daemon=True).start()
        done = 0
        while done < len(readers):
            s = q.get()
            if s is end:
                done += 1
            else:
                yield s
    return reader


import sys as _sys  # noqa: E402
# `paddle.reader.decorator.<fn>` is the reference's spelling of the same functions
decorator = _sys.modules[__name__]
_sys.modules[__name__ + ".decorator"] = decorator
