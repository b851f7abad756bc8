"""DCNv2 ``_ext`` backend on the MI355X engine.

Drop-in for the CUDA extension that ``codes/models/modules/DCNv2/setup.py`` builds and
``codes/models/modules/DCNv2/dcn_v2.py:11`` imports (``import _ext as _backend``): put this
directory ahead of the compiled ``_ext`` on ``sys.path`` (or ``PYTHONPATH``) and the reference's
own ``dcn_v2.py`` -- ``_DCNv2``, ``dcn_v2_conv``, ``DCNv2``, ``DCN``, ``DCN_sep`` -- runs unchanged
on ``stif_dcn_v2_forward`` / ``stif_dcn_v2_backward`` (include/stif.h), training included (the
autograd ``_DCNv2.backward`` calls ``dcn_v2_backward``).  PSROI pooling is not provided (STIF does
not use ``DCNv2Pooling``).
"""
import os
import sys

_REPO = os.environ.get("STIF_AMD_REPO") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _REPO not in sys.path:
    sys.path.insert(0, _REPO)

import stif_pkg  # noqa: E402

_stif = stif_pkg.load()

# vision.cpp:4 -- same arguments (input, weight, bias, offset, mask, kernel_h, kernel_w, stride_h,
# stride_w, pad_h, pad_w, dilation_h, dilation_w, deformable_group), returns a new NCHW tensor
dcn_v2_forward = _stif.ops.dcn_v2_forward


# vision.cpp:5 -- (input, weight, bias, offset, mask, grad_output, kernel_h, kernel_w, stride_h,
# stride_w, pad_h, pad_w, dilation_h, dilation_w, deformable_group) -> [grad_input, grad_offset,
# grad_mask, grad_weight, grad_bias]
dcn_v2_backward = _stif.ops.dcn_v2_backward


def dcn_v2_psroi_pooling_forward(*args, **kwargs):
    """vision.cpp:6 -- DCNv2Pooling is not used by STIF."""
    raise NotImplementedError("dcn_v2_psroi_pooling_forward is not provided by stif_amd")


def dcn_v2_psroi_pooling_backward(*args, **kwargs):
    """vision.cpp:7."""
    raise NotImplementedError("dcn_v2_psroi_pooling_backward is not provided by stif_amd")
