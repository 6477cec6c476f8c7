"""Voice conversion over a decode directory: the
reference's `vae_npvc.decoder.basic.Decoder` (decoder/basic.py:10-86) on this
package's model and Kaldi writer.

`decode(decode_dir, output_dir)` reads `trials` (utt, target speaker(s)),
`feats.scp` and optionally `spk2spk_id`, converts every trial with
`model.infer((feat (1, mel, T), target (1, 1)))` and writes the converted
(T, mel) features to `output_dir/feats.{ark,scp}` as Kaldi compressed matrices
(compression_method=1, as the reference, :52-53).  Unlike the reference
(:31-37) there is no silent CPU retry: the model runs on the MI355X through
libvqx or raises.
"""
import logging
from importlib import import_module
from pathlib import Path

import numpy as np
import torch

from ..dataset.kaldi_io import WriteHelper, load_mat

logger = logging.getLogger()


class Decoder(object):
    def __init__(self, config):
        model_type = config.get("model_type", "vae_npvc_amd.model.vqvae:Model").split(":")
        if not config.get("use_gpu", True):
            raise RuntimeError("vae_npvc_amd decodes on the MI355X only (use_gpu: false is not supported)")
        self.device = torch.device("cuda")
        module = import_module(model_type[0], package=None)
        model_name = "Model" if len(model_type) < 2 else model_type[1]
        self.model = getattr(module, model_name)(config).to(self.device)
        self.model.eval()

    def decode_step(self, feat, spk):
        with torch.no_grad():
            return self.model.infer((feat, spk))

    def decode(self, decode_dir, output_dir, compress=True):
        decode_dir = Path(decode_dir)
        output_dir = str(output_dir)
        for file in ["trials", "feats.scp"]:
            if not (decode_dir / file).is_file():
                raise FileNotFoundError(f"No such file {decode_dir / file}")
        trials = [line.strip().split(None, 1) for line in open(decode_dir / "trials") if line.strip()]
        feats_scp = dict(line.strip().split(None, 1) for line in open(decode_dir / "feats.scp") if line.strip())
        spk2spk_id = None
        if (decode_dir / "spk2spk_id").exists():
            spk2spk_id = dict(line.strip().split(None, 1) for line in open(decode_dir / "spk2spk_id") if line.strip())
        wspecifier = "ark,scp:{0}/feats.ark,{0}/feats.scp".format(output_dir)
        with WriteHelper(wspecifier, compression_method=1 if compress else None) as wf:
            for i, (utt, target) in enumerate(trials):
                logger.info(f"Decode {i}: {utt} to {target}")
                feat = torch.from_numpy(np.array(load_mat(feats_scp[utt]))).float().to(self.device)
                feat = feat.t().unsqueeze(0)
                if spk2spk_id:
                    target = [int(spk2spk_id[t]) for t in target.split()]
                else:
                    target = [int(t) for t in target.split()]
                if len(target) != 1:
                    raise ValueError(f"trial {utt}: one target speaker per utterance, got {target}")
                target = torch.tensor(target).long().to(self.device).view(1, -1)
                feat_decode = self.decode_step(feat, target)
                wf[utt] = feat_decode[0].t().detach().cpu().numpy()

    def get_model_info(self):
        return self.model

    def load_checkpoint(self, checkpoint_file):
        checkpoint_data = torch.load(checkpoint_file, map_location="cpu", weights_only=True)
        self.model.load_state_dict(checkpoint_data["model"])
        return checkpoint_data["iteration"]
