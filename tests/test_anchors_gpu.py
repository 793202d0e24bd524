"""Rows a18-a20 on the GPU: anchors bit-exact, targets' masks/indices bit-exact, encoded and
decoded boxes within 2 ulp-level tolerance (transcendentals) of the numpy oracle."""
import numpy as np
import pytest
import torch

from oracle import ref_anchors as RA
from tf2mv_amd.anchors import Anchors

pytestmark = pytest.mark.gpu
ASPECTS = [(1.0, 1.0), (1.4, 0.7), (0.7, 1.4)]


@pytest.mark.parametrize("args", [(0, 0, (10, 10), 3, [(1.0, 1.0)], 3.0), (3, 7, (512, 512), 3, ASPECTS, 4.0),
                                  (3, 7, (640, 640), 3, ASPECTS, 4.0), (3, 7, (128, 128), 3, ASPECTS, 4.0)])
def test_anchor_boxes_bit_exact(args):
    a = Anchors(*args)
    ref = RA.generate_boxes(*args)
    for got, want in zip(a.boxes, ref):
        np.testing.assert_array_equal(got.cpu().numpy(), want)


def synthetic_gt(rng, B, G, size):
    boxes = np.zeros((B, G, 4), np.float32)
    cls = np.zeros((B, G), np.int32)
    n = rng.integers(1, G + 1, B).astype(np.int32)
    for b in range(B):
        for k in range(n[b]):
            s = np.exp(rng.uniform(np.log(16), np.log(size * 0.8)))
            ar = rng.uniform(0.5, 2.0)
            h, w = s * np.sqrt(ar), s / np.sqrt(ar)
            cy, cx = rng.uniform(0, size, 2)
            boxes[b, k] = [cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2]
            cls[b, k] = rng.integers(1, 81)
    return boxes.astype(np.float32), cls, n


@pytest.mark.parametrize("size,B", [(128, 3), (512, 2)])
def test_generate_targets_and_decode(size, B):
    rng = np.random.default_rng(size)
    a = Anchors(3, 7, (size, size), 3, ASPECTS, 4.0)
    ref_levels = RA.generate_boxes(3, 7, (size, size), 3, ASPECTS, 4.0)
    G = 9
    boxes, cls, n = synthetic_gt(rng, B, G, size)
    # add the test_anchors style exact hit: a GT equal to an anchor
    boxes[0, 0] = ref_levels[0][3, 5, 4]
    t = a.generate_targets_batched(torch.tensor(boxes), torch.tensor(cls), torch.tensor(n))
    pyr = t.pyr
    tb, tc, tm = t.box.cpu().numpy(), t.cls.cpu().numpy(), t.mask.cpu().numpy()
    npos = 0
    for b in range(B):
        ob, oc, om, oi = RA.generate_targets(ref_levels, boxes[b, : n[b]], cls[b, : n[b]], 81)
        for s, (H, W) in enumerate(a.level_sizes):
            sl = pyr.seg_slice(s)
            rows = slice(sl.start + b * H * W, sl.start + (b + 1) * H * W)
            np.testing.assert_array_equal(tm[rows].reshape(H, W, 9), om[s][..., 0].astype(np.uint8))
            np.testing.assert_array_equal(tc[rows].reshape(H, W, 9), oi[s])
            np.testing.assert_allclose(tb[rows].reshape(H, W, 9, 4), ob[s], rtol=2e-6, atol=1e-6)
            npos += int(om[s].sum())
    assert npos > 0
    # decode of the encoded targets returns the GT box of every positive anchor (a20)
    dec = a.convert_outputs_boxes(t.box.view(pyr.rows, 36), pyr=pyr, ld=36)
    for s, (H, W) in enumerate(a.level_sizes):
        d = dec[s].cpu().numpy()
        enc = tb[pyr.seg_slice(s)].reshape(B, H, W, 9, 4)
        want = RA.decode(ref_levels[s][None], enc).astype(np.float64)
        # ulp-level bound: each coordinate is center -/+ size/2 computed in fp32 (the GPU may
        # fuse ty*ha+ya and uses a 1-ulp expf), so allow 4 ulp of |center| + |size|/2
        ctr_y, ctr_x = (want[..., 0] + want[..., 2]) / 2, (want[..., 1] + want[..., 3]) / 2
        hh, ww = (want[..., 2] - want[..., 0]) / 2, (want[..., 3] - want[..., 1]) / 2
        mag_y, mag_x = np.abs(ctr_y) + np.abs(hh), np.abs(ctr_x) + np.abs(ww)
        tol = 4 * np.finfo(np.float32).eps * np.stack([mag_y, mag_x, mag_y, mag_x], -1)
        err = np.abs(d.astype(np.float64) - want)
        assert (err <= tol).all(), (float((err / tol).max()), float(err.max()))


def test_reference_format_roundtrip():
    rng = np.random.default_rng(1)
    a = Anchors(0, 0, (10, 10), 3, [(1.0, 1.0)], 3.0)
    ob, oc, om = a.generate_targets(torch.tensor([[3, 3, 6, 6], [5, 5, 9, 9]], dtype=torch.float32),
                                    torch.tensor([1, 2]), 3)
    assert bool(om[0][4, 4, 0, 0]) and oc[0][4, 4, 0].tolist() == [0, 1, 0]
    assert ob[0][4, 4, 0].abs().max().item() == 0.0


@pytest.mark.parametrize("dt,size,NC", [("f32", 128, 5), ("bf16", 128, 5), ("f32", 256, 81)])
def test_detect_nms_matches_oracle(dt, size, NC):
    """§8(f) row 2: convert_outputs_one + DIoU-NMS (anchors.py:161-202, nms.py:5-61) on the GPU.
    Kept boxes, their order and class ids bit-exact with the oracle's literal sort/boolean_mask
    loop on the same decoded boxes and logits; scores (sigmoid) within 2 ulp."""
    from tf2mv_amd.runtime import Pyr
    rng = np.random.default_rng(size + NC)
    a = Anchors(3, 7, (size, size), 3, ASPECTS, 4.0, device="cuda")
    A, B = 9, 3
    pyr = a.pyramid(B)
    tdt = torch.float32 if dt == "f32" else torch.bfloat16
    ld_b, ld_c = A * 4, A * NC + 7  # an unaligned logits stride, like inference's A*NC
    rel = torch.zeros(pyr.rows, ld_b)
    logits = torch.zeros(pyr.rows, ld_c)
    for s in range(pyr.nseg):
        sl = pyr.seg_slice(s)
        n = pyr.seg_rows(s)
        rel[sl] = torch.tensor(rng.normal(0, 0.3, (n, ld_b)), dtype=torch.float32)
        # logits with exact ties and many background winners
        lg = np.round(rng.normal(0, 2, (n, ld_c)) * 4) / 4
        logits[sl] = torch.tensor(lg, dtype=torch.float32)
    rel_g, log_g = rel.to("cuda", tdt), logits.to("cuda", tdt)
    box_levels, cls_levels = [], []
    for s, (fh, fw) in enumerate(a.level_sizes):
        sl = pyr.seg_slice(s)
        box_levels.append(rel_g[sl].view(B, fh, fw, A, 4))
        cls_levels.append(log_g[sl, : A * NC].view(B, fh, fw, A, NC))
    dec = a.convert_outputs_boxes(tuple(box_levels))
    ob, oc, os_, cnt = a.detect(dec, tuple(cls_levels))
    torch.cuda.synchronize()
    for b in range(B):
        rb, rc, rs = RA.convert_outputs_one([d[b].cpu().numpy() for d in dec],
                                            [c[b].float().cpu().numpy() for c in cls_levels])
        k = int(cnt[b])
        assert k == len(rb) and k > 0
        np.testing.assert_array_equal(ob[b, :k].cpu().numpy(), rb)
        np.testing.assert_array_equal(oc[b, :k].cpu().numpy(), rc)
        np.testing.assert_allclose(os_[b, :k].cpu().numpy(), rs, rtol=3e-7, atol=0)
    # the single-image API of the reference
    bb, cc, ss = a.convert_outputs_one(1, dec, tuple(cls_levels))
    assert bb.shape[0] == int(cnt[1])


def test_label_file_pipeline_targets_match_oracle(tmp_path):
    """§8(f) row 4 end to end: the committed reference-format label file -> load_labels ->
    prepare (proportional resize, clip, 2-px filter, field order) -> collate ->
    generate_targets_batched on the GPU, masks/indices bit-exact against the oracle run on the
    same prepared boxes."""
    import os
    from PIL import Image
    from tf2mv_amd import data as D
    fix = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)).save(tmp_path / "img_a.png")
    Image.fromarray(rng.integers(0, 256, (640, 480, 3), dtype=np.uint8)).save(tmp_path / "img_b.png")
    classes = D.load_classes(os.path.join(fix, "classes.txt"))
    labels = D.load_labels(os.path.join(fix, "labels.txt"), str(tmp_path), classes, log=lambda *a: None)[:2]
    size = 512
    a = Anchors(3, 7, (size, size), 3, ASPECTS, 4.0)
    samples = [D.prepare(l, (size, size)) for l in labels]
    x, gb, gc, n = D.collate(samples, "cuda")
    assert x.shape == (2, size, size, 3) and x.is_cuda
    t = a.generate_targets_batched(gb, gc, n)
    ref_levels = RA.generate_boxes(3, 7, (size, size), 3, ASPECTS, 4.0)
    tc, tm = t.cls.cpu().numpy(), t.mask.cpu().numpy()
    npos = 0
    for b, (_, boxes, cls) in enumerate(samples):
        _, _, om, oi = RA.generate_targets(ref_levels, boxes, cls, len(classes))
        for s, (H, W) in enumerate(a.level_sizes):
            sl = t.pyr.seg_slice(s)
            rows = slice(sl.start + b * H * W, sl.start + (b + 1) * H * W)
            np.testing.assert_array_equal(tm[rows].reshape(H, W, 9), om[s][..., 0].astype(np.uint8))
            np.testing.assert_array_equal(tc[rows].reshape(H, W, 9), oi[s])
            npos += int(om[s].sum())
    assert npos > 0
