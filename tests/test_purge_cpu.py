"""@purge (PartitionRuntimeImpl.java:120-147, 346-402) on the CPU: the QL front end's annotation rules and
the oracle's restatement against the reference's own PartitionDataPurgingTestCase.

The reference test sends six events, sleeps 1100 ms and sends two more; its purge task (interval and
idle.period 1 s, scheduled by every initPartition call) cleans IBM, whose last event is more than 1 s old
at some task time, so IBM's length(3) window starts over (avg 100.0, not 200.0).  On the app clock the six
sends are 1 ms apart (the wall-clock spacing the reference's strict `lastSeen + idle < now` relies on)."""
import pytest

from oracle.pyoracle import OracleApp
from siddhi_amd import ql

APP = ("define stream streamA (symbol string, price int);"
       "@purge(enable='true', interval='1 sec', idle.period='1 sec') "
       "partition with (symbol of streamA) begin @info(name = 'query1') "
       "from streamA#window.length(3) select symbol, avg(price) as total insert into StockQuote ; end ")


def test_partition_data_purging_kat():
    # PartitionDataPurgingTestCase.java:52-126 (expected values :78-103)
    o = OracleApp(APP)
    o.add_stream_callback("StockQuote")
    o.start()
    evs = [("IBM", 100), ("IBM", 100), ("IBM", 400), ("WSO2", 40), ("WSO2", 10), ("WSO2", 10), ("IBM", 100),
           ("WSO2", 10)]
    for t, e in zip([0, 1, 2, 3, 4, 5, 1100, 1101], evs):
        o.set_time(t)
        o.send("streamA", list(e), ts=t)
    rows = [r for cb in o.outputs() for r in cb["in"]]
    assert [r[1] for r in rows] == [100.0, 100.0, 200.0, 40.0, 25.0, 20.0, 100.0, 10.0]
    assert [r[0] for r in rows] == ["IBM"] * 3 + ["WSO2"] * 3 + ["IBM", "WSO2"]


def test_without_purge_the_window_carries_on():
    o = OracleApp(APP.replace("enable='true'", "enable='false'"))
    o.add_stream_callback("StockQuote")
    o.start()
    for t, e in zip([0, 1, 2, 1100], [("IBM", 100), ("IBM", 100), ("IBM", 400), ("IBM", 100)]):
        o.set_time(t)
        o.send("streamA", list(e), ts=t)
    assert [r[1] for cb in o.outputs() for r in cb["in"]] == [100.0, 100.0, 200.0, 200.0]


def test_purge_descriptor_fields():
    d = ql.compile_app(APP)
    q = d["queries"][0]
    assert q["purge"] == {"interval": 1000, "idle": 1000} and q["partition_id"] == 0
    d = ql.compile_app(APP.replace(" interval='1 sec',", ""))
    assert d["queries"][0]["purge"] == {"interval": 300000, "idle": 1000}   # default interval
    assert "purge" not in ql.compile_app(APP.replace("enable='true'", "enable='false'"))["queries"][0]


@pytest.mark.parametrize("ann,msg", [("@purge(interval='1 sec', idle.period='1 sec') ", "missing element 'enable'"),
                                     ("@purge(enable='yes', idle.period='1 sec') ", "Invalid value for enable"),
                                     ("@purge(enable='true', interval='1 sec') ", "missing element 'idle.period'"),
                                     ("@purge(enable='true', idle.period='1 fortnight') ", "does not exists")])
def test_purge_annotation_errors(ann, msg):
    src = APP.replace("@purge(enable='true', interval='1 sec', idle.period='1 sec') ", ann)
    with pytest.raises(ql.SiddhiParserError, match=msg):
        ql.compile_app(src)
