"""pyhocon-compatible config accessor + the GASFM model confs.

The reference passes a pyhocon ConfigTree (main.py:80-87) and the model only
calls ``get_int / get_bool / get_string(key, default=...)`` on it
(graph_attn_sfm.py:12-41, baseNet.py:12-14).  pyhocon is not installed
offline, so ``Conf`` provides the same accessors over a nested dict, plus a
parser for the flat/nested ``key = value`` / ``key { ... }`` subset of HOCON
the reference's conf files use.  A real pyhocon ConfigTree works unchanged.

Presets restate the ``model`` sections of
  confs/gasfm/learning_euc_rhaug-15-20_gasfm.conf:43-75  (12 blocks)
  confs/gasfm/optim_euc_gasfm.conf:9-38                  (9 blocks)
"""
import copy
import re

_MISSING = object()


class Conf:
    def __init__(self, d=None):
        self.d = d if d is not None else {}

    def _get(self, key, default):
        cur = self.d
        for part in key.split("."):
            if not isinstance(cur, dict) or part not in cur:
                if default is _MISSING:
                    raise KeyError(f"config key '{key}' missing")
                return default
            cur = cur[part]
        return cur

    def get(self, key, default=_MISSING):
        return self._get(key, default)

    def get_int(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else int(v)

    def get_float(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else float(v)

    def get_bool(self, key, default=_MISSING):
        v = self._get(key, default)
        if isinstance(v, str):
            return v.lower() in ("true", "yes", "on", "1")
        return None if v is None else bool(v)

    def get_string(self, key, default=_MISSING):
        v = self._get(key, default)
        return None if v is None else str(v)

    def put(self, key, value):
        cur = self.d
        parts = key.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = value
        return self

    @classmethod
    def parse_string(cls, text):
        """Parse the HOCON subset used by confs/*.conf (no includes/substitutions)."""
        text = re.sub(r"(?m)^\s*(#|//).*$", "", text)
        toks = re.findall(r'"(?:[^"\\]|\\.)*"|[{}\[\]=:,\n]|[^\s{}\[\]=:,"]+', text)
        pos = 0

        def value(tok):
            if tok.startswith('"'):
                return tok[1:-1]
            low = tok.lower()
            if low in ("true", "false"):
                return low == "true"
            if low == "null":
                return None
            try:
                return int(tok)
            except ValueError:
                try:
                    return float(tok)
                except ValueError:
                    return tok

        def skip_nl():
            nonlocal pos
            while pos < len(toks) and toks[pos] in ("\n", ","):
                pos += 1

        def parse_list():
            nonlocal pos
            out = []
            while True:
                skip_nl()
                if toks[pos] == "]":
                    pos += 1
                    return out
                if toks[pos] == "{":
                    pos += 1
                    out.append(parse_obj(True))
                else:
                    out.append(value(toks[pos]))
                    pos += 1

        def parse_obj(braced):
            nonlocal pos
            out = {}
            while True:
                skip_nl()
                if pos >= len(toks):
                    return out
                if toks[pos] == "}":
                    pos += 1
                    return out
                key = toks[pos].strip('"')
                pos += 1
                if toks[pos] in ("=", ":"):
                    pos += 1
                if toks[pos] == "{":
                    pos += 1
                    val = parse_obj(True)
                elif toks[pos] == "[":
                    pos += 1
                    val = parse_list()
                else:
                    val = value(toks[pos])
                    pos += 1
                cur = out
                parts = key.split(".")
                for p in parts[:-1]:
                    cur = cur.setdefault(p, {})
                if isinstance(val, dict) and isinstance(cur.get(parts[-1]), dict):
                    cur[parts[-1]].update(val)
                else:
                    cur[parts[-1]] = val

        return cls(parse_obj(False))

    @classmethod
    def parse_file(cls, path):
        with open(path) as f:
            return cls.parse_string(f.read())


_GASFM_MODEL = {
    "type": "graph_attn_sfm.GraphAttnSfMNet",
    "n_heads": 4,
    "stateful_global_features": True,
    "global2view_and_global2scenepoint_enabled": False,
    "n_feat_proj": 32,
    "n_feat_scenepoint": 64,
    "n_feat_view": 1024,
    "n_feat_global": 2048,
    "num_layers": 12,
    "n_hidden_layers_scenepoint_update": 0,
    "n_hidden_layers_view_update": 0,
    "n_hidden_layers_global_update": 0,
    "n_hidden_layers_proj_update": 0,
    "use_norm_proj_update": True,
    "add_residual_skipconn_proj_update": True,
    "add_skipconn_from_init_projfeat": True,
    "pos_emb_n_freq": 0,
    "depth_head": {"enabled": False, "n_feat": 128, "n_hidden_layers": 2},
    "view_head": {"enabled": True, "n_hidden_layers": 2, "rot_representation": "quat"},
    "scenepoint_head": {"enabled": True, "n_hidden_layers": 2},
}


def learning_conf(**model_overrides):
    """learning_euc_rhaug-15-20_gasfm.conf model section (12 blocks)."""
    m = copy.deepcopy(_GASFM_MODEL)
    m.update(model_overrides)
    return Conf({"dataset": {"calibrated": True}, "model": m})


def optim_conf(**model_overrides):
    """optim_euc_gasfm.conf model section (9 blocks)."""
    m = copy.deepcopy(_GASFM_MODEL)
    m["num_layers"] = 9
    m.update(model_overrides)
    return Conf({"dataset": {"calibrated": True}, "model": m})


def small_conf(num_layers=2, **model_overrides):
    """Reduced widths for fast parity tests (SURVEY.md §8(c) fixture (ii))."""
    m = copy.deepcopy(_GASFM_MODEL)
    m.update({"num_layers": num_layers, "n_feat_view": 64, "n_feat_global": 128})
    m.update(model_overrides)
    return Conf({"dataset": {"calibrated": True}, "model": m})
