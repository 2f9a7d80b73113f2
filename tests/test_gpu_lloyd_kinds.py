"""Lloyd pass kinds are exact: with every bounded pass forced to kTile, or to
kQueue, or to kList (twice), or the default mix, the fits equal the plain Lloyd E-step every pass
(MW_LLOYD_NOBOUND) bit for bit — labels, centers, n_iter — for k = 8..20 in
one batched launch, and repeated runs agree.  Regression: the queue pass
gathers only the F floats of each row into LDS, and the scaled-row read
took the padded pair of the tile's last row from LDS no pass had written
(NaN * 0 = NaN): a few labels per pass changed from run to run."""
import contextlib
import os
import sys

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu


def _rows():
    import milwrm_amd as M
    from milwrm_amd import device as D

    raw, mask = D.synth_slide(1536, 1536, 30, seed=20251015, mode="hard")
    im = M.img.from_device(raw, mask)
    with contextlib.redirect_stdout(sys.stderr):
        est, pix = im.calculate_non_zero_mean()
        df = pd.DataFrame({"Img": [im], "batch_names": ["b"], "mean estimators": [est],
                           "pixels": [pix]})
        lab = M.mxif_labeler(df)
        lab.prep_cluster_data(features=list(range(30)), sigma=2, fract=0.2)
    return lab._rows


@pytest.mark.timeout(300)
def test_pass_kinds_equal_full_estep(gpu, monkeypatch):
    from milwrm_amd import kmeans as KM

    rows = _rows()
    ks = list(range(8, 21))
    out = {}
    for name, qb, qk, nobound in [("full", -1.0, KM.KIND_QUEUE, True), ("tile", -1.0, KM.KIND_QUEUE, False),
                                  ("queue", 2.0, KM.KIND_QUEUE, False), ("queue_again", 2.0, KM.KIND_QUEUE, False),
                                  ("list", 2.0, KM.KIND_LIST, False),
                                  ("list_again", 2.0, KM.KIND_LIST, False),
                                  ("default", KM.QUEUE_BELOW, KM.QUEUE_KIND, False)]:
        monkeypatch.setattr(KM, "QUEUE_BELOW", qb)
        monkeypatch.setattr(KM, "QUEUE_KIND", qk)
        if nobound:
            monkeypatch.setenv("MW_LLOYD_NOBOUND", "1")
        else:
            monkeypatch.delenv("MW_LLOYD_NOBOUND", raising=False)
        with contextlib.redirect_stdout(sys.stderr):
            fits = KM.fit_many(rows, ks, random_state=18)
        out[name] = [(np.asarray(m.labels_).copy(), m.cluster_centers_.copy(), m.n_iter_) for m in fits]
    for name in ("tile", "queue", "queue_again", "list", "list_again", "default"):
        for i, k in enumerate(ks):
            a, b = out["full"][i], out[name][i]
            assert a[2] == b[2], f"k={k} {name}: n_iter {b[2]} vs {a[2]}"
            np.testing.assert_array_equal(b[0], a[0], err_msg=f"k={k} {name} labels")
            np.testing.assert_array_equal(b[1], a[1], err_msg=f"k={k} {name} centers")
