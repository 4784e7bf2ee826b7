"""Streaming ingest (read_methylation_data, src/data.cpp:116-153 +
compute_markers_statistics :233-283): a marker-major fp64 file larger than
the 256 MB staging buffers, with ragged N, read by several threads, lands in
HBM bit for bit; the statistics match the oracle."""
import numpy as np
import pytest

from conftest import relerr

pytestmark = pytest.mark.gpu

va = pytest.importorskip("vampomi_amd")
from oracle import pyoracle as O  # noqa: E402  (checker)


@pytest.mark.parametrize("threads", ["1", "5"])
def test_multichunk_file_ingest(tmp_path, monkeypatch, threads):
    monkeypatch.setenv("VAMPOMI_IO_THREADS", threads)
    N, Mt = 4099, 20011  # 656 MB: three staging chunks, the last one partial
    X = O.generate_markers(31, 1, N, 0, Mt)
    p = tmp_path / "big.bin"
    X.tofile(p)
    with va.Data(N, Mt) as d:
        d.read_methylation_data(str(p))
        for i0 in (0, 8180, 8181, 16362, Mt - 3):
            assert np.array_equal(d.get_meth_data(i0, 3), X[i0:i0 + 3])
        mo, so = O.marker_stats(X)
        assert relerr(d.get_mave(), mo) < 1e-13 and relerr(d.get_msig(), so) < 1e-13


def test_short_file_is_an_error(tmp_path):
    N, Mt = 100, 50
    p = tmp_path / "short.bin"
    np.zeros((Mt - 1) * N).tofile(p)
    with va.Data(N, Mt) as d:
        with pytest.raises(va.VampomiError) as e:
            d.read_methylation_data(str(p))
        assert e.value.status == 4
