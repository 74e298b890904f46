"""ReLU-sparse row images (rvx_row_image_pack, rvx_sage_forward_exchange3; rvx.h): a GraphSAGE
layer's output is (n + s).max(0.0) (crates/ruvector-postgres/src/gnn/graphsage.rs:172-176), so
about half of every row is +0.0; the next layer's overlapped gather reads the neighbour rows
from a packed image (3 KiB slot: bitmap + the other values) instead of the dense table.

Bars: the image holds every row bit for bit (decoded here in numpy), and a stack run with
images is bit-identical to the same stack without them — same terms, same order — on the
chunked/helped pipeline (RVX_SAGE_CHUNKS; a layer is chunked from 16384 rows per chunk), with and without the carried normalisation, with
rows the image cannot hold (more than 736 values other than +0.0: dense fallback), empty
neighbourhoods, rows of more than 64 neighbours, -0.0 and NaN entries."""
import ctypes

import numpy as np
import pytest

import oracle as O
import ruvector_amd as rv
from ruvector_amd import _lib as L

pytestmark = pytest.mark.gpu

SLOT, CAP = 3072, 736


def decode_image(img: np.ndarray, n: int, dim: int):
    """numpy reader of the image layout (kernels.hpp RowImage): column c = 256 j + 4 lane + k
    is held iff bit 4j + k of the lane's u16 is set; held values follow in column order. Rows
    the image does not hold (nnz > CAP) come back as NaN."""
    slots = img[: n * SLOT].reshape(n, SLOT)
    nnz = img[n * SLOT: n * SLOT + 2 * n].view(np.uint16)
    c = np.arange(dim)
    lane, j, k = (c % 256) // 4, c // 256, c % 4
    out = np.full((n, dim), np.nan, np.float32)
    for r in np.nonzero(nnz <= CAP)[0]:
        h = slots[r, :128].view(np.uint16).astype(np.uint32)
        mask = ((h[lane] >> (4 * j + k)) & 1).astype(bool)
        assert mask.sum() == nnz[r]
        row = np.zeros(dim, np.float32)
        row[mask] = slots[r, 128:].view(np.float32)[: nnz[r]]
        out[r] = row
    return out, nnz


def _stack(layers, g, x, n, defer, images):
    off = np.array([0, n], np.int64)
    off_p = off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    xb = rv.Buffer.from_numpy(x)
    d1, d2 = layers[0].out_features, layers[1].out_features
    t1, t2, iv = rv.Buffer(n * d1 * 4), rv.Buffer(n * d2 * 4), rv.Buffer(n * 4)
    img = rv.row_image(n, d1) if images else None
    L.call("rvx_sage_forward_exchange3", layers[0]._h, g.handle, xb.handle, None, None, t1.handle,
           iv.handle if defer else None, img.handle if img else None, off_p, None, 0)
    y1 = t1.download(np.float32, (n, d1))
    L.call("rvx_sage_forward_exchange3", layers[1]._h, g.handle, t1.handle, iv.handle if defer else None,
           img.handle if img else None, t2.handle, None, None, off_p, None, 0)
    raw = img.download(np.uint8, (rv.row_image_bytes(n, d1),)) if img else None
    return y1, t2.download(np.float32, (n, d2)), raw


def _graph(n, deg, seed):
    rng = np.random.default_rng(seed)
    degs = rng.integers(0, 2 * deg + 1, n)
    degs[::17] = 0
    degs[5::101] = 3 * 64 + 7  # rows of more than 64 neighbours
    rp = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    col = rng.integers(0, n, int(rp[-1])).astype(np.int32)
    return rp, col


@pytest.mark.parametrize("img_reg", ["1", "0"])  # expansion in registers (default) or through LDS windows
@pytest.mark.parametrize("defer", [True, False])
@pytest.mark.parametrize("dims,n,deg,chunks", [((768, 768, 768), 70000, 9, 4), ((256, 640, 512), 50000, 6, 3),
                                               ((768, 768, 256), 34000, 12, 2)])
def test_sage_stack_with_row_image_is_bit_identical(monkeypatch, defer, dims, n, deg, chunks, img_reg):
    monkeypatch.setenv("RVX_SAGE_CHUNKS", str(chunks))
    monkeypatch.setenv("RVX_IMG_REG", img_reg)
    d0, d1, d2 = dims
    x = O.fill_uniform(n * d0, 400 + n).reshape(n, d0) - 0.5
    rp, col = _graph(n, deg, 401)
    g = rv.Graph.from_csr(rp, col)
    layers = [rv.GraphSAGELayer(d0, d1, num_samples=4 * 64), rv.GraphSAGELayer(d1, d2, num_samples=4 * 64)]
    y1a, y2a, _ = _stack(layers, g, x, n, defer, False)
    y1b, y2b, raw = _stack(layers, g, x, n, defer, True)
    assert np.array_equal(y1a.view(np.uint32), y1b.view(np.uint32))
    assert np.array_equal(y2a.view(np.uint32), y2b.view(np.uint32))
    # the image holds layer 1's rows bit for bit (a sample of rows), and most of them fit
    rows = np.arange(0, n, max(1, n // 300))
    dec, nnz = decode_image(raw, n, d1)
    assert np.array_equal(nnz.astype(np.int64), (y1b.view(np.uint32) != 0).sum(axis=1))
    held = rows[nnz[rows] <= CAP]
    assert len(held) > 0.9 * len(rows) and nnz.mean() < 0.75 * d1  # ReLU zeros
    assert np.array_equal(dec[held].view(np.uint32), y1b[held].view(np.uint32))


@pytest.mark.parametrize("img_reg", ["1", "0"])
def test_row_image_dense_fallback_signed_zeros_and_nan(monkeypatch, img_reg):
    """An input table packed directly (rvx_row_image_pack): rows with every value nonzero (the
    dense fallback), rows of mixed density, an all-zero row, -0.0 and NaN entries. A layer
    reading it through x_image gives the bits of the layer reading the table."""
    monkeypatch.setenv("RVX_SAGE_CHUNKS", "3")
    monkeypatch.setenv("RVX_IMG_REG", img_reg)
    n, d, deg = 50000, 768, 10
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((n, d)) * 0.1).astype(np.float32)
    keep = rng.random((n, d)) < rng.choice([0.2, 0.5, 0.7, 0.95, 1.0], n)[:, None]
    x = np.where(keep, x, np.float32(0.0)).astype(np.float32)
    x[3] = 0.0
    x[4, ::7] = -0.0
    x[11, 5] = np.nan
    rp, col = _graph(n, deg, 8)
    g = rv.Graph.from_csr(rp, col)
    layer = rv.GraphSAGELayer(d, 512, num_samples=4 * 64)
    xb = rv.Buffer.from_numpy(x)
    img = rv.row_image(n, d)
    rv.pack_row_image(xb, n, d, img, 0, n // 2)
    rv.pack_row_image(xb, n, d, img, n // 2)
    raw = img.download(np.uint8, (rv.row_image_bytes(n, d),))
    dec, nnz = decode_image(raw, n, d)
    assert np.array_equal(nnz.astype(np.int64), (x.view(np.uint32) != 0).sum(axis=1))
    held = nnz <= CAP
    assert 0.4 < held.mean() < 0.9 and held[3] and held[4]
    assert np.array_equal(dec[held].view(np.uint32), x[held].view(np.uint32))

    off = np.array([0, n], np.int64)
    off_p = off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    outs = []
    for im in (None, img):
        y = rv.Buffer(n * 512 * 4)
        L.call("rvx_sage_forward_exchange3", layer._h, g.handle, xb.handle, None, im.handle if im else None,
               y.handle, None, None, off_p, None, 0)
        outs.append(y.download(np.float32, (n, 512)))
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


def test_row_image_argument_checks():
    with pytest.raises(rv.RvxError):
        rv.row_image_bytes(10, 256)  # the image is for 512 < dim <= 768
    n, d = 1000, 768
    xb = rv.Buffer(n * d * 4)
    small = rv.Buffer(rv.row_image_bytes(n, d) - 4)
    with pytest.raises(rv.RvxError):
        rv.pack_row_image(xb, n, d, small)
    img = rv.row_image(n, d)
    with pytest.raises(rv.RvxError):
        rv.pack_row_image(xb, n, d, img, 10, n)  # past the table
