"""CPU oracle for the RE⫶TR hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from this package, and only as the checker (or the timed CPU baseline).
The product path (``retr_amd``) never imports it and has no CPU fallback.

Contents
--------
``tv_resnet``  restatement of torchvision's ResNet-{18,34,50,101} (third-party dependency of
               the reference, absent from this image, version unpinned — the reference uses the
               ``weights=`` API so torchvision >= 0.13).  Also used as
               the ``torchvision`` stand-in that lets ``tests/golden/make_golden.py`` import the
               reference's own ``models.caption``.
``model``      functional fp32 CPU restatement of ``Caption.forward`` + CE + ``greedy`` that
               follows the reference op order (file:line cited per function).

Parity pinning: ``model`` is checked against golden vectors produced by running the reference
modules themselves (``/root/reference``) in the build container (tests/golden/*.npz, script
``tests/golden/make_golden.py``).  The transformer half, head, loss and decode loop are pinned
by the reference code directly.  The conv stack is torchvision arithmetic: it is pinned to
torchvision's documented layer semantics only (parity for torchvision internals is
"unpinned").
"""
