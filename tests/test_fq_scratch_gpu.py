"""ibwa_fq_share_scratch: ingest contexts of one device parsing in turn through one parse scratch
(the CLI's slots) keep their own kept reads -- each context's staged batch aligns as its own block
did -- and ibwa_fq_offset refuses a block whose line table another context has parsed over."""
import ctypes as c

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fastq(rng, n, L):
    recs = []
    for i in range(n):
        s = "".join(rng.choice(list("ACGT"), L))
        recs.append(f"@r{i}\n{s}\n+\n{'I' * L}\n")
    return "".join(recs).encode()


def _parse(L, ctx, raw):
    n_rec, consumed, not_strict = c.c_int64(), c.c_uint64(), c.c_int()
    cap = len(raw) // 48 + 17
    lens = (c.c_int32 * cap)()
    buf = c.create_string_buffer(raw, len(raw))
    rc = L.ibwa_fq_parse(ctx, buf, len(raw), 0, 0, c.byref(n_rec), c.byref(consumed), c.byref(not_strict), lens, None,
                         cap)
    assert rc == 0, L.ibwa_last_error()
    return n_rec.value, list(lens[:n_rec.value])


def test_shared_scratch_keeps_each_block():
    from ibwa_amd import engine as E
    L = E.lib()
    rng = np.random.default_rng(3)
    a_raw, b_raw = _fastq(rng, 300, 40), _fastq(rng, 500, 25)
    a, b = c.c_void_p(), c.c_void_p()
    assert L.ibwa_ctx_create(0, c.byref(a)) == 0 and L.ibwa_ctx_create(0, c.byref(b)) == 0
    try:
        assert L.ibwa_fq_share_scratch(b, a) == 0
        assert L.ibwa_fq_share_scratch(b, b) != 0
        na, la = _parse(L, a, a_raw)
        off = c.c_uint64()
        assert L.ibwa_fq_offset(a, 10, c.byref(off)) == 0
        assert off.value == a_raw.index(b"@r10\n")
        nb, lb = _parse(L, b, b_raw)
        assert (na, nb) == (300, 500) and set(la) == {40} and set(lb) == {25}
        # a's line table is gone (b parsed over the shared scratch) ...
        assert L.ibwa_fq_offset(a, 10, c.byref(off)) != 0
        assert L.ibwa_fq_offset(b, 7, c.byref(off)) == 0 and off.value == b_raw.index(b"@r7\n")
        # ... but its kept reads are its own
        ka, kb = c.c_int64(), c.c_int64()
        L.ibwa_fq_stats(a, c.byref(ka), None)
        L.ibwa_fq_stats(b, c.byref(kb), None)
        assert (ka.value, kb.value) == (300, 500)
        x = c.c_void_p()
        assert L.ibwa_ctx_create(0, c.byref(x)) == 0
        try:
            assert L.ibwa_batch_stage_fq(x, a, 0, 300, 40) == 0
            assert L.ibwa_batch_stage_fq(x, b, 0, 500, 25) == 0
            assert L.ibwa_batch_stage_fq(x, a, 0, 301, 40) != 0
        finally:
            L.ibwa_ctx_destroy(x)
    finally:
        L.ibwa_ctx_destroy(b)
        L.ibwa_ctx_destroy(a)
