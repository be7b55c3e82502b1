"""Generates tests/golden/ref_fec.json from the reference's own sources, read as text (run in the
build container, where /root/reference exists; the GPU box never reads it). Data only: the code-
block size column of TS 36.212 Table 5.1.3-3 as the reference lists it (tc_cb_sizes,
lib/src/sections_part3/fix/cbsegm.cpp:34-46 -- that file needs srsRAN headers, so it cannot be
compiled here) and the FEC constants of pcc_enc.cpp:37-46 and pdc_enc.cpp:36."""
import json
import os
import re

REF = os.environ.get("REF", "/root/reference")
here = os.path.dirname(os.path.abspath(__file__))
cb = open(os.path.join(REF, "lib/src/sections_part3/fix/cbsegm.cpp")).read()
body = re.search(r"tc_cb_sizes\[[^\]]*\]\s*=\s*\{([^}]*)\}", cb).group(1)
sizes = [int(x) for x in re.findall(r"\d+", body)]
pcc = open(os.path.join(REF, "lib/src/phy/fec/pcc_enc.cpp")).read()
pdc = open(os.path.join(REF, "lib/src/phy/fec/pdc_enc.cpp")).read()


def const(src, name):
    return int(re.search(r"\b" + name + r"\s*=\s*(0x[0-9A-Fa-f]+|\d+)", src).group(1), 0)


fx = {"tc_cb_sizes": sizes,
      "pcc": {n: const(pcc, n) for n in ("crc_bits", "SRSRAN_PDSCH_MAX_TDEC_ITERS", "mask_none", "mask_mimo_cl",
                                          "mask_bf", "mask_mimo_cl_bf", "pcc_g_init")},
      "pdc": {"SRSRAN_PDSCH_MAX_TDEC_ITERS": const(pdc, "SRSRAN_PDSCH_MAX_TDEC_ITERS")}}
json.dump(fx, open(os.path.join(here, "ref_fec.json"), "w"), indent=1)
print(len(sizes), fx["pcc"], fx["pdc"])
