"""ORACLE — CPU restatement of the JABD reference hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import anything from here, and only as the
checker (or the timed CPU baseline).  The product package never imports it.

Parity status:
  * The reference (/root/reference/JABD2080ti) is pure Python and may not be
    imported or executed in this pipeline (environment denial recorded in
    SURVEY.md §8c).  Every function here is restated from the reference text
    and cites the file:line it follows.
  * Pinned by the reference's own known answer: the anchor count printed by
    utils/anchors.py:104-105 (29518 for steps 8/16/32/64 at 840²) plus
    hand-derived counts; hand-made KATs for NMS and match (ties, shared best
    prior, IoU exactly at the threshold) are committed in tests/.
  * torchvision.ops.nms (third-party, absent here, version unpinned) is
    restated from its published CPU algorithm in nms_ref.c.
  * Everything else (model forward, losses, encodings) is PARITY UNPINNED:
    no reference-generated vectors exist; the restatement follows the
    reference text op-for-op in PyTorch-CPU fp32.
"""
