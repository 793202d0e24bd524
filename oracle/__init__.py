"""CPU oracle for the EfficientDet hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The product path
(``tensorflow2-machine-vision_amd/``) never imports it and has no CPU fallback.

Contents
  * ``ref_model``   — torch-CPU restatement (fp64 by default) of the reference's
                      EfficientDet forward, loss and train step (TF semantics: asymmetric
                      SAME padding, training-mode BN, Keras loss reductions).
  * ``ref_anchors`` — numpy fp32 restatement of anchors / IoU / target encoding / decoding.

Pinning.  TensorFlow is absent here and on the GPU box, so the TF-op semantics the
restatement encodes are *parity unpinned* by the reference's own tests
(which are print-only).  What IS pinned: (1) shape/config arithmetic against fixtures made
by importing the reference's TF-free helpers (tests/golden/make_golden.py), (2) the
anchor/IoU known-answer tests derivable from tests/test_anchors.py and iou.py:103-112.
"""
