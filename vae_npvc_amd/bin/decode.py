#!/usr/bin/env python3
"""Conversion driver: the reference's bin/decode.py:21-76 (decoder type from
the YAML, checkpoint load, `Decoder.decode(decode_dir, output_dir)`).

  python -m vae_npvc_amd.bin.decode -c conf.yaml --checkpoint ckpt \\
      --decode-dir data/eval --output-dir out
"""
import argparse
import logging
import os
from importlib import import_module
from pathlib import Path

import numpy as np
import torch
import yaml


def decode(args):
    output_dir = Path(args.output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    config = yaml.safe_load(open(args.config))
    config.update({"use_gpu": args.gpu[0] != "c"})
    decoder_type = config.get("decoder_type", "vae_npvc_amd.decoder.basic:Decoder").split(":")
    seed = config.get("seed", 777)
    np.random.seed(seed)
    torch.manual_seed(seed)
    module = import_module(decoder_type[0], package=None)
    decoder = getattr(module, "Decoder" if len(decoder_type) < 2 else decoder_type[1])(config)
    if args.checkpoint is None:
        raise ValueError("--checkpoint is required")
    decoder.load_checkpoint(args.checkpoint)
    logger = logging.getLogger()
    logger.setLevel(logging.INFO)
    logger.addHandler(logging.FileHandler(filename=str(output_dir / "decode.log")))
    logger.info("Decoding dataset: {}".format(args.decode_dir))
    decoder.decode(args.decode_dir, output_dir)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("-c", "--config", type=str, required=True)
    p.add_argument("--output-dir", type=str, required=True)
    p.add_argument("--checkpoint", type=str, default=None)
    p.add_argument("--decode-dir", type=str, required=True)
    p.add_argument("-g", "--gpu", type=str, default="0")
    args = p.parse_args(argv)
    if args.gpu[0] != "c":
        os.environ["HIP_VISIBLE_DEVICES"] = args.gpu
    decode(args)


if __name__ == "__main__":
    main()
