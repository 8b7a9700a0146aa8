"""Write tests/golden/descriptors/*.json: version-1 app descriptors (include/siddhi_gfx_descriptor.schema.json)
of the BASELINE configs and a few boundary cases, so the C-ABI tests can create apps from the descriptor
alone, the way the Java shim does, without the Python QL front end.

    python tests/golden/make_descriptors.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from siddhi_amd import synth  # noqa: E402
from siddhi_amd.ql import compile_app  # noqa: E402

S = synth.STOCK_STREAM
CASES = {
    "config1": synth.CONFIG1_QL,
    "config2": synth.CONFIG2_QL,
    "config3": synth.CONFIG3_QL,
    "config4": synth.CONFIG4_QL,
    "config5": synth.CONFIG5_FULL_QL,
    # one lowered query and one that is not (a pattern inserting expired events): the app is created and
    # the second query reports SG_E_UNSUPPORTED with its reasons
    "partial": S + " @info(name='ok') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] "
                   "within 1 sec select e1.symbol, e2.price insert into Out;"
                   " @info(name='agg') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] "
                   "select e1.symbol, sum(e2.price) as total group by e1.symbol insert expired events into Out2;",
}


def main():
    for name, ql in CASES.items():
        with open(os.path.join(HERE, "descriptors", name + ".json"), "w") as f:
            json.dump(compile_app(ql), f, indent=1)
    print("wrote", len(CASES))


if __name__ == "__main__":
    main()
