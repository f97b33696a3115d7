"""Test infrastructure (not product code): the forward an UNMODIFIED reference ``FoundationStereo`` runs after ``patch_reference``.

``patch_reference(core.foundation_stereo)`` rebinds the reference module's star-imported names to
this package, but the reference's own ``forward`` / ``upsample_disp`` bodies stay
in charge: they call the unfused volume build (``build_gwc_volume`` + ``proj_cmb`` +
``build_concat_volume`` + ``cat``), run ``corr_stem`` / ``corr_feature_att`` / ``classifier`` as plain
module calls (so ``corr_stem[0]``, ``proj_cmb`` and the classifier's ``Conv3d(14, 1, 7)`` -- built from
``torch.nn`` in the reference's ``__init__`` -- stay on MIOpen), compute the context after the volume
path, and step ``update_block`` once per iteration with no stream overlap.

``forward_reference_order`` restates that control flow statement for statement
(``core/foundation_stereo.py:183-191`` and ``:194-254``) over this package's ``FoundationStereo``
instance, whose module tree and ``state_dict`` are the reference's.  It is what the drop-in seam
executes on a GPU box, where the reference itself does not exist; ``tests/test_gpu_reference_order.py``
holds it to the reference goldens and the oracle, and ``tools/reference_order_bench.py`` times it
beside the fused ``FoundationStereo.forward``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from foundationstereo_amd.foundation_stereo import autocast, normalize_image
from foundationstereo_amd.geometry import Combined_Geo_Encoding_Volume
from foundationstereo_amd.submodule import build_concat_volume, build_gwc_volume, context_upsample, disparity_regression


def upsample_disp_reference_order(model, disp, mask_feat_4, stem_2x):
    """core/foundation_stereo.py:183-191."""
    with autocast(model.args.mixed_precision):
        xspx = model.spx_2_gru(mask_feat_4, stem_2x)
        spx_pred = model.spx_gru(xspx)
        spx_pred = F.softmax(spx_pred, 1)
        up_disp = context_upsample(disp * 4., spx_pred).unsqueeze(1)
    return up_disp.float()


def forward_reference_order(model, image1, image2, iters=12, flow_init=None, test_mode=False, low_memory=False,
                            init_disp=None):
    """core/foundation_stereo.py:194-254 over ``model`` (a ``foundationstereo_amd`` FoundationStereo)."""
    B = len(image1)
    low_memory = low_memory or (model.args.get('low_memory', False))
    image1 = normalize_image(image1)
    image2 = normalize_image(image2)
    with autocast(model.args.mixed_precision):
        out, vit_feat = model.feature(torch.cat([image1, image2], dim=0))
        vit_feat = vit_feat[:B]
        features_left = [o[:B] for o in out]
        features_right = [o[B:] for o in out]
        stem_2x = model.stem_2(image1)

        gwc_volume = build_gwc_volume(features_left[0], features_right[0], model.args.max_disp // 4, model.cv_group)
        left_tmp = model.proj_cmb(features_left[0])
        right_tmp = model.proj_cmb(features_right[0])
        concat_volume = build_concat_volume(left_tmp, right_tmp, maxdisp=model.args.max_disp // 4)
        del left_tmp, right_tmp
        comb_volume = torch.cat([gwc_volume, concat_volume], dim=1)
        comb_volume = model.corr_stem(comb_volume)
        comb_volume = model.corr_feature_att(comb_volume, features_left[0])
        comb_volume = model.cost_agg(comb_volume, features_left)

        prob = F.softmax(model.classifier(comb_volume).squeeze(1), dim=1)
        if init_disp is None:
            init_disp = disparity_regression(prob, model.args.max_disp // 4)

        cnet_list = model.cnet(image1, vit_feat=vit_feat, num_layers=model.args.n_gru_layers)
        cnet_list = list(cnet_list)
        net_list = [torch.tanh(x[0]) for x in cnet_list]
        inp_list = [torch.relu(x[1]) for x in cnet_list]
        inp_list = [model.cam(x) * x for x in inp_list]
        att = [model.sam(x) for x in inp_list]

    geo_fn = Combined_Geo_Encoding_Volume(features_left[0].float(), features_right[0].float(), comb_volume.float(),
                                          num_levels=model.args.corr_levels, dx=model.dx)
    b, c, h, w = features_left[0].shape
    coords = torch.arange(w, dtype=torch.float, device=init_disp.device).reshape(1, 1, w, 1).repeat(b, h, 1, 1)
    disp = init_disp.float()
    disp_preds = []

    for itr in range(iters):
        disp = disp.detach()
        geo_feat = geo_fn(disp, coords, low_memory=low_memory)
        with autocast(model.args.mixed_precision):
            net_list, mask_feat_4, delta_disp = model.update_block(net_list, inp_list, geo_feat, disp, att)

        disp = disp + delta_disp.float()
        if test_mode and itr < iters - 1:
            continue

        disp_up = upsample_disp_reference_order(model, disp.float(), mask_feat_4.float(), stem_2x.float())
        disp_preds.append(disp_up)

    if test_mode:
        return disp_up

    return init_disp, disp_preds
