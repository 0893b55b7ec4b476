"""Checkpoint (.ckpt = torch.save(state_dict)) round trip between the drop-in plugins and the
reference-layout modules (the oracle restatements carry the reference's module tree): every
plugin's state_dict loads strictly into its reference counterpart and back, through a file read
with torch.load(weights_only=True).  CPU only — no forward pass."""
import importlib

import pytest
import torch

from oracle import models as OM

PAIRS = [("mfcc_bgru", OM.MfccBGRU), ("fbanks_cnn", OM.FbanksCNN), ("spec_bgru", OM.SpecBGRU),
         ("resnet_bgru", OM.ResnetBGRU), ("mfrn_bgru", OM.MfrnBGRU), ("cnn_bgru", OM.CnnBGRU),
         ("spec_cnn", OM.SpecCNN), ("analyst", OM.Analyst)]


@pytest.mark.parametrize("name,ocls", PAIRS)
def test_ckpt_round_trip(tmp_path, name, ocls):
    mod = importlib.import_module("speechrecognitionproject_amd.models.model_" + name)
    ours = mod.Network()
    ref = ocls()
    # reference layout -> file -> plugin
    sd = OM.seeded_state_dict(ref, seed=3)
    torch.save(sd, tmp_path / "ref.ckpt")
    ours.load_state_dict(torch.load(tmp_path / "ref.ckpt", weights_only=True), strict=True)
    for k, v in ours.state_dict().items():
        assert torch.equal(v, sd[k]), k
    # plugin -> file -> reference layout
    torch.save(ours.state_dict(), tmp_path / "ours.ckpt")
    ref2 = ocls()
    ref2.load_state_dict(torch.load(tmp_path / "ours.ckpt", weights_only=True), strict=True)
    for k, v in ref2.state_dict().items():
        assert torch.equal(v, sd[k]), k
