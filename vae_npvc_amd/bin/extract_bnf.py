#!/usr/bin/env python3
"""Bottleneck-feature (codebook index) extraction: the reference's
bin/extract_bnf.py:22-67 on this package's model and Kaldi I/O.

  python -m vae_npvc_amd.bin.extract_bnf -c conf.yaml --model_path ckpt \\
      --bnf_kind id|csid|token [--output_txt true] RSPECIFIER WSPECIFIER

`id`: one codebook index per frame; `csid`: consecutive duplicates merged;
`token`: the (T, 1) index column.  Text output writes `utt <i><j>...` lines,
otherwise a Kaldi archive of int32 vectors (WSPECIFIER `ark:...` or
`ark,scp:...`).
"""
import argparse
import os
from importlib import import_module

import numpy as np
import torch
import yaml

from ..dataset.kaldi_io import ReadHelper, WriteHelper


def extract_bnf(args):
    output_txt = args.output_txt.lower() in ["true"]
    config = yaml.safe_load(open(args.config))
    model_type = config.get("model_type", "vae_npvc_amd.model.vqvae").split(":")
    module = import_module(model_type[0], package=None)
    model = getattr(module, "Model" if len(model_type) < 2 else model_type[1])(config)
    if args.model_path:
        model.load_state_dict(torch.load(args.model_path, map_location="cpu", weights_only=True)["model"])
    model.cuda().eval()
    if output_txt and args.bnf_kind in ["id", "csid"]:
        writer = open(args.wspecifier, "w")
    else:
        writer = WriteHelper(args.wspecifier)
        output_txt = False
    n = 0
    for utt, feat in ReadHelper(args.rspecifier):
        feat_in = torch.from_numpy(np.array(feat)).float().cuda().t().unsqueeze(0)
        with torch.no_grad():
            bnf = model.encode(feat_in).unsqueeze(-1)          # (1, T, 1)
        if args.bnf_kind == "id":
            out = bnf.view(-1).cpu().numpy()
        elif args.bnf_kind == "csid":
            out = bnf.view(-1).unique_consecutive().cpu().numpy()
        elif args.bnf_kind == "token":
            out = bnf[0].cpu().numpy()
        else:
            raise ValueError(f"unknown bnf_kind {args.bnf_kind!r}")
        if output_txt:
            writer.write("{} {}\n".format(utt, "".join("<{}>".format(b) for b in out.reshape(-1))))
        else:
            writer.write(utt, out.astype(np.int32))
        n += 1
    writer.close()
    return n


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-c", "--config", type=str, required=True)
    p.add_argument("--model_path", type=str, default=None)
    p.add_argument("--bnf_kind", type=str, default="id")
    p.add_argument("--output_txt", type=str, default="true")
    p.add_argument("--gpu", type=str, default=None)
    p.add_argument("rspecifier", type=str)
    p.add_argument("wspecifier", type=str)
    args = p.parse_args(argv)
    if args.gpu is not None:
        os.environ["HIP_VISIBLE_DEVICES"] = args.gpu
    return extract_bnf(args)


if __name__ == "__main__":
    main()
