"""The CPU restatement (oracle/) against the reference's own known answers.

Each fixture is a TestNG case transcribed from the reference test suites
(tests/golden/extract_kats.py, reviewed in tests/golden/review_kats.py).  Passing all of them
is what pins the oracle before it is trusted as the parity checker for the HIP path.
"""
import pytest

from kat import check, load_kats, run_app
from oracle.pyoracle import OracleApp

KATS = load_kats()


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_oracle_matches_reference_kat(kat):
    if kat["expect"].get("create_error"):      # @Test(expectedExceptions = SiddhiAppCreationException)
        with pytest.raises(Exception):
            OracleApp(kat["app"])
        return
    outs = run_app(OracleApp(kat["app"]), kat)
    assert check(kat, outs) == []
