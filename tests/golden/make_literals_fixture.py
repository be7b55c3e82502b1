"""Generates tests/golden/ref_literals.json from the reference's own sources, read as text (run in the
build container, where /root/reference exists; the GPU box never reads it). Data only: the literal
tables of sections_part3 that the oracle (oracle/oracle_tables.cpp), the product's host geometry
(csrc/host/geometry.cpp, exported by dnrp_query_table) and the kernels' constants restate. These
files need srsRAN / VOLK headers (stf.cpp, transmit_diversity_precoding.cpp) or are plain literal
tables, so they are pinned by extraction instead of compilation:

  W_1 .. W_6, j                    beamforming_and_antenna_port_mapping.cpp:250-286, .hpp:83-86
  N_TS_N_TX_idx / _codebook_index_max / _codebook_index_nonzero   beamforming_...mapping.hpp:88-119
  scaling_factor_optimal_DAC       beamforming_and_antenna_port_mapping.cpp:146-186 (statements)
  y_b_1, y_b_2, y_b_4 (STF)        stf.cpp:161-169
  cover_sequence (active branch)   stf.hpp:146-151
  y_b_1 (DRS, 56 complex)          drs.hpp:124-135
  index_N_TS_x, pattern_minus_1_j_1_j   transmit_diversity_precoding.cpp:37-75
"""
import json
import math
import os
import re

REF = os.environ.get("REF", "/root/reference")
SP3 = os.path.join(REF, "lib/src/sections_part3")
INC = os.path.join(REF, "lib/include/dectnrp/sections_part3")
here = os.path.dirname(os.path.abspath(__file__))


def read(*p):
    return open(os.path.join(*p)).read()


bf = read(SP3, "beamforming_and_antenna_port_mapping.cpp")
bfh = read(INC, "beamforming_and_antenna_port_mapping.hpp")
J = int(re.search(r"static constexpr int8_t j\s*=\s*(\d+)\s*;", bfh).group(1))


def w_entry(tok):
    tok = tok.strip()
    return {"j": J, "-j": -J}.get(tok, None) if "j" in tok else int(tok)


W = {}
for m in re.finditer(r"const common::vec2d<int8_t> W_t::W_(\d)\s*=\s*\{(.*?)\};", bf, flags=re.S):
    rows = re.findall(r"\{([^{}]*)\}", m.group(2))
    W[f"W_{m.group(1)}"] = [[w_entry(t) for t in r.split(",") if t.strip()] for r in rows]
assert sorted(W) == [f"W_{i}" for i in range(1, 7)], sorted(W)


def array2d(name):
    body = re.search(name + r"\s*=\s*\{\s*\{(.*?)\}\s*\};", bfh, flags=re.S).group(1)
    return [[int(x) for x in re.findall(r"-?\d+", r)] for r in re.findall(r"\{([^{}]*)\}", "{" + body + "}")]


tables = {n: array2d(n) for n in ("N_TS_N_TX_idx", "N_TS_N_TX_codebook_index_max", "N_TS_N_TX_codebook_index_nonzero")}


def fexpr(e):
    """'1.0f' or '1.0f / std::sqrt(2.0f)' as written in the reference (float arithmetic)."""
    e = e.strip()
    m = re.fullmatch(r"1\.0f(?:\s*/\s*std::sqrt\((\d+\.\d+)f\))?", e)
    assert m, e
    import numpy as np
    return float(np.float32(1.0) / np.sqrt(np.float32(float(m.group(1))))) if m.group(1) else 1.0


# scaling_factor_optimal_DAC: replay the constructor's statements in source order
sec = bf[bf.index("scaling_factor_optimal_DAC.push_back(std::vector<float>())"):]
sec = sec[:sec.index("dectnrp_assert(scaling_factor_optimal_DAC.size()")]
opt = [[] for _ in range(7)]
pat = re.compile(r"for \(uint32_t i = 0; i < (\d+); \+\+i\) \{\s*scaling_factor_optimal_DAC\[(\d)\]\.push_back\(([^;]*)\);\s*\}"
                 r"|scaling_factor_optimal_DAC\[(\d)\]\.push_back\(([^;]*)\);"
                 r"|scaling_factor_optimal_DAC\[(\d)\]\s*=\s*std::vector<float>\{([^}]*)\};", flags=re.S)
for m in pat.finditer(sec):
    if m.group(1):
        opt[int(m.group(2))] += [fexpr(m.group(3))] * int(m.group(1))
    elif m.group(4):
        opt[int(m.group(4))].append(fexpr(m.group(5)))
    else:
        opt[int(m.group(6))] = [fexpr(x) for x in re.split(r",(?![^(]*\))", m.group(7)) if x.strip()]

stf = read(SP3, "stf.cpp")
y_stf = {f"y_b_{b}": [int(float(x)) for x in re.findall(r"-?\d+",
                                                        re.search(r"stf_t::y_b_%d\s*=\s*\{([^}]*)\}" % b, stf).group(1))]
         for b in (1, 2, 4)}
stfh = read(INC, "stf.hpp")
cov = re.search(r"cover_sequence\{\s*#ifdef SECTIONS_PART_3_STF_COVER_SEQUENCE_ACTIVE(.*?)#else", stfh, flags=re.S).group(1)
cover = [float(x) for x in re.findall(r"-?\d+\.\d+", cov)]

drsh = read(INC, "drs.hpp")
body = re.search(r"y_b_1\[56\]\s*=\s*\{(.*?)\};", drsh, flags=re.S).group(1)
drs_y = [[int(a), int(b)] for a, b in re.findall(r"\{\s*(-?\d+)\s*,\s*(-?\d+)\s*\}", body)]

td = read(SP3, "transmit_diversity_precoding.cpp")
idx = [[], [], []]
for r, a, b in re.findall(r"index_N_TS_x\[(\d)\]\.push_back\(std::vector<uint32_t>\{(\d+),\s*(\d+)\}\)", td):
    idx[int(r)].append([int(a), int(b)])
pattern = [[float(a), float(b)] for a, b in re.findall(r"pattern_minus_1_j_1_j\[i(?: \+ 1)?\]\s*=\s*cf_t\{(-?\d+\.\d+)f,\s*(-?\d+\.\d+)f\}", td)]
modulo = {int(n): int(v) for n, v in re.findall(r"case (\d+):\s*return (\d+);", td)}
modulo.setdefault(8, int(re.search(r"// N_TS == 8\s*return (\d+);", td).group(1)))

fx = {"j": J, **W, **tables, "scaling_factor_optimal_DAC": opt, **{"stf_" + k: v for k, v in y_stf.items()},
      "cover_sequence": cover, "drs_y_b_1": drs_y, "index_N_TS_x": idx, "pattern_minus_1_j_1_j": pattern,
      "txdiv_modulo": {str(k): v for k, v in sorted(modulo.items())}}
assert [len(W[f"W_{i}"]) for i in range(1, 7)] == [6, 28, 3, 22, 5, 1]
assert [len(o) for o in opt] == [1, 6, 28, 3, 22, 5, 1], [len(o) for o in opt]
assert len(drs_y) == 56 and len(cover) == 9 and [len(r) for r in idx] == [1, 6, 12]
json.dump(fx, open(os.path.join(here, "ref_literals.json"), "w"), indent=None, separators=(",", ":"))
print({k: (len(v) if isinstance(v, (list, dict)) else v) for k, v in fx.items()})
