"""Import harness for the reference's hot-path modules (THIS container only).

Test infrastructure, not product code: used solely by ``oracle/make_golden.py``
to run the reference's own PyTorch modules on synthetic weights and record
golden vectors into ``tests/golden/``.  Nothing on the GPU box imports this
file (``/root/reference`` does not exist there).

Recipe: SURVEY.md Appendix B.  The package-level ``import onmt`` fails because
torchtext is absent (``onmt/__init__.py:4``), so empty parent packages are
registered and each hot-path module is loaded by file path.  ``translate/
translator.py`` gets stub modules for its non-hot-path imports.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

REF = os.environ.get("NANODEC_REFERENCE", "/root/reference")
_LOADED = {}


def _pkg(name, path=None):
    if name in sys.modules:
        return sys.modules[name]
    m = types.ModuleType(name)
    m.__path__ = [path] if path else []
    sys.modules[name] = m
    return m


def _load(name, rel):
    if name in sys.modules and getattr(sys.modules[name], "__file__", None):
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


def load_reference():
    """Returns a namespace with the reference classes used by the golden
    generator.  Raises if the reference tree is missing."""
    if _LOADED:
        return _LOADED["ns"]
    if not os.path.isdir(REF):
        raise FileNotFoundError(f"reference tree not found at {REF}")
    sys.dont_write_bytecode = True
    for n, p in [("onmt", "onmt"), ("onmt.modules", "onmt/modules"), ("onmt.utils", "onmt/utils"),
                 ("onmt.encoders", "onmt/encoders"), ("onmt.models", "onmt/models"),
                 ("encoder", "encoder"), ("decoder", "decoder")]:
        m = _pkg(n, os.path.join(REF, p))
        if "." in n:
            parent, child = n.rsplit(".", 1)
            setattr(sys.modules[parent], child, m)
    mha = _load("onmt.modules.multi_headed_attn", "onmt/modules/multi_headed_attn.py")
    sys.modules["onmt.modules"].MultiHeadedAttention = mha.MultiHeadedAttention
    _load("onmt.modules.position_ffn", "onmt/modules/position_ffn.py")
    aan = _load("onmt.modules.average_attn", "onmt/modules/average_attn.py")
    sys.modules["onmt.modules"].AverageAttention = aan.AverageAttention
    util_class = _load("onmt.modules.util_class", "onmt/modules/util_class.py")
    sys.modules["onmt.modules"].Elementwise = util_class.Elementwise
    emb = _load("onmt.modules.embeddings", "onmt/modules/embeddings.py")
    misc = _load("onmt.utils.misc", "onmt/utils/misc.py")
    sys.modules["onmt.utils"].misc = misc
    _load("onmt.utils.rnn_factory", "onmt/utils/rnn_factory.py")
    _load("onmt.encoders.encoder", "onmt/encoders/encoder.py")
    enc_t = _load("encoder.transformer", "encoder/transformer.py")
    enc_n = _load("encoder.nano_encoder", "encoder/nano_encoder.py")
    dec_t = _load("decoder.transformer", "decoder/transformer.py")

    # --- translate/translator.py with stubbed non-hot-path imports ---------
    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__path__ = []
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    # onmt/translate/{penalties,beam}.py for the classic (non --fast) Beam path
    _pkg("onmt.translate", os.path.join(REF, "onmt/translate"))
    sys.modules["onmt"].translate = sys.modules["onmt.translate"]
    pen = _load("onmt.translate.penalties", "onmt/translate/penalties.py")
    sys.modules["onmt.translate"].penalties = pen
    beam = _load("onmt.translate.beam", "onmt/translate/beam.py")
    sys.modules["onmt.translate"].beam = beam
    sys.modules["onmt.translate"].Beam = beam.Beam
    sys.modules["onmt.translate"].GNMTGlobalScorer = beam.GNMTGlobalScorer
    for name in ("configargparse", "matplotlib", "matplotlib.pyplot", "models", "models.model_builder",
                 "models.opts", "utils", "utils.labelop", "translate", "translate.translation",
                 "onmt.decoders", "onmt.decoders.ensemble"):
        if name not in sys.modules:
            stub(name)
    sys.modules["utils.labelop"].extract_fast5_raw = None
    stub("inputters")
    stub("inputters.inputter", make_features=lambda b, side, data_type="text": getattr(b, side))
    sys.modules["inputters"].inputter = sys.modules["inputters.inputter"]
    sys.modules["translate.translation"].TranslationBuilder = object
    translator = _load("translate.translator", "translate/translator.py")

    ns = types.SimpleNamespace(
        TransformerEncoder=enc_t.TransformerEncoder,
        NanoEncoder=enc_n.NanoEncoder,
        TransformerDecoder=dec_t.TransformerDecoder,
        Embeddings=emb.Embeddings,
        Translator=translator.Translator,
        GNMTGlobalScorer=beam.GNMTGlobalScorer,
        tile=misc.tile,
    )
    _LOADED["ns"] = ns
    return ns
