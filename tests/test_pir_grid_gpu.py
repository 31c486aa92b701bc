"""The reference's dense-PIR benchmark grid on the GPU scan, against the
oracle: pir/dense_dpf_pir_database_benchmark.cc:125-157
(BM_BatchedInnerProductOnVariableSizeValues) times InnerProductWith on
2^20 records of 32 / 256 / 2,048 / 16,384 bytes on average — each record's
size drawn from [avg - 8, avg + 8) (GenerateRandomStringsVariableSize,
pir/testing/mock_pir_database.cc:83-101) — at batches of 1, 2, 10 and 100.

Here the two wide sizes (2,048 and 16,384 B: rows of 129 / 1,025 16-byte
words, the KPirScanG G = 1 slices and KPirScanM4's row staging) run at the
grid's record count with a ragged last tile (2^20 - 45 records: the last
128-record selection block is partial, and its bits past the end are set),
built through the bulk variable-size insert (dpf_amd_pir_db_insert_packed,
Builder::Insert per record), stored at whole 128-byte lines per row.
Selections are random inside three 4,096-record windows (the first, one in
the middle, the last reaching the ragged end) and
zero elsewhere, so the oracle (inner_product_hwy.cc:270-296) checks the
windows' records while the scan streams the whole table; records outside the
windows are a non-periodic pattern, so a row leaking into a sum would show.
The 32 / 256 B shapes are covered by tests/test_api_gpu.py and the c4 tests.
"""
import numpy as np
import pytest

from oracle import pyoracle as po

pytestmark = pytest.mark.gpu

N = (1 << 20) - 45
WINDOW = 4096
MAX_SIZE_DIFF = 8  # kMaxSizeDiff, dense_dpf_pir_database_benchmark.cc:35


@pytest.fixture(scope="module", params=[2048, 16384], ids=["avg2048", "avg16384"])
def grid_db(request, cuda):
    import torch
    from distributed_point_functions_amd import pir as P
    avg = request.param
    rng = np.random.default_rng(avg)
    # absl::Uniform(bitgen, -diff, diff) is half-open: [avg - 8, avg + 8)
    sizes = avg + rng.integers(-MAX_SIZE_DIFF, MAX_SIZE_DIFF, N)
    offs = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(sizes, out=offs[1:])
    total = int(offs[-1])
    period = (1 << 20) + 7  # coprime with every record size: no two rows alike
    base = np.frombuffer(rng.bytes(period), dtype=np.uint8)
    data = np.empty(total, dtype=np.uint8)
    reps = total // period
    data[:reps * period].reshape(reps, period)[:] = base
    data[reps * period:] = base[:total - reps * period]
    windows = [(0, WINDOW), ((N // 2) // 128 * 128, (N // 2) // 128 * 128 + WINDOW),
               ((N - WINDOW) // 128 * 128, N)]
    for s, e in windows:
        data[offs[s]:offs[e]] = np.frombuffer(rng.bytes(int(offs[e] - offs[s])), dtype=np.uint8)
    db = P.DenseDpfPirDatabase()
    db.insert_packed(data, sizes).build()
    d = dict(avg=avg, db=db, sizes=sizes, offs=offs, data=data, windows=windows)
    yield d
    d.clear()
    del db
    torch.cuda.empty_cache()


def device_row_stride(max_size):
    """The database's row stride (csrc/pir.cc DeviceRowStride): the
    reference's 16-byte alignment (dense_dpf_pir_database.cc:40-52), padded
    to whole 128-byte lines when that costs at most 1/16 more bytes."""
    s16 = max(16, (max_size + 15) // 16 * 16)
    s128 = (s16 + 127) // 128 * 128
    return s128 if (s128 - s16) * 16 <= s16 else s16


def test_grid_database_layout(grid_db):
    """Wide rows start on a cache line; results are as long as the largest
    value (inner_product_hwy.cc:252-256)."""
    db, sizes = grid_db["db"], grid_db["sizes"]
    assert db.size == N
    assert db.max_value_size == int(sizes.max())
    assert db.record_stride == device_row_stride(int(sizes.max()))
    assert db.record_stride % 128 == 0


@pytest.mark.parametrize("q", [1, 2, 10, 100])
def test_grid_inner_product_matches_oracle_on_windows(grid_db, q):
    db, offs, data = grid_db["db"], grid_db["offs"], grid_db["data"]
    nb = (N + 127) // 128
    rng = np.random.default_rng(q * 7 + grid_db["avg"])
    sel = np.zeros((q, nb, 2), dtype=np.uint64)
    for s, e in grid_db["windows"]:
        b0, b1 = s // 128, (e + 127) // 128
        sel[:, b0:b1] = rng.integers(0, 1 << 63, size=(q, b1 - b0, 2), dtype=np.uint64) * 2 + \
            rng.integers(0, 2, size=(q, b1 - b0, 2), dtype=np.uint64)
    assert sel[:, nb - 1, 1].any()  # bits past the last record are set
    got = db.inner_product_with(sel)
    m = db.max_value_size
    recs = [data[offs[i]:offs[i + 1]].tobytes() for s, e in grid_db["windows"] for i in range(s, e)]
    blocks = [[int(w[0]) | (int(w[1]) << 64)
               for s, e in grid_db["windows"] for w in sel[k, s // 128:(e + 127) // 128]]
              for k in range(q)]
    want = po.inner_product(recs, blocks)
    assert len(got) == q
    for k in range(q):
        w = want[k] + b"\0" * (m - len(want[k]))
        assert len(got[k]) == m
        assert got[k] == w, "query %d of %d" % (k, q)
