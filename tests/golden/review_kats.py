"""Reviewed subset of the auto-transcribed fixtures: kats_auto.json -> kats.json.

Every exclusion carries its reason.  Excluded cases exercise features outside the hot-path scope
(joins, scalar functions, stddev, partition inner streams) or assert a
creation-time exception rather than outputs.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

EXCLUDE = {
    # @Test(expectedExceptions = SiddhiAppCreationException.class): not output fixtures
    "CountPatternTestCase.testQuery14": "scalar function instanceOfFloat (out of scope: executor/function)",
    "SequenceTestCase.testQuery20_1": "multi-value select of a count state (MultiValueVariableFunctionExecutor) not restated yet",
    "SequenceTestCase.testQuery20_2": "scalar function ifThenElse (out of scope: executor/function)",
    "PatternPartitionTestCase.testPatternPartitionQuery32": "partition inner stream (#Stream) out of scope",
    "PatternPartitionTestCase.testPatternPartitionQuery33": "partition inner stream (#Stream) out of scope",
    "LengthWindowTestCase.lengthWindowTest4": "stddev aggregator out of scope (SURVEY.md §2 row A15: OUT)",
    "LengthBatchWindowTestCase.lengthBatchWindowTest8": "join (out of scope)",
    "LengthBatchWindowTestCase.lengthBatchWindowTest9": "join (out of scope)",
    "LengthBatchWindowTestCase.lengthBatchWindowTest13": "join (out of scope)",
    "LengthBatchWindowTestCase.lengthBatchWindowTest14": "join (out of scope)",
}
EXCLUDE.update({
    "CountPatternTestCase.testQuery16": "multi-value select `e2.price` of the <2:> count state (OBJECT-typed "
                                        "List output, as SequenceTestCase.testQuery20_1; unpinned)",
    "CountPatternTestCase.testQuery21": "multi-value select `e1.price as prices` (OBJECT-typed List output: no "
                                        "column encoding in the C ABI; unpinned)",
    "GroupByTestCase.testGroupByQuery2": "timeBatch window (out of scope: SURVEY.md §2 windows row)",
    "WindowPartitionTestCase.testWindowPartitionQuery3": "scalar function default (out of scope: executor/function)",
    "WindowPartitionTestCase.testWindowPartitionQuery5": "timeBatch window (out of scope: SURVEY.md §2 windows row)",
})


# In-callback assertions transcribed by hand (extract_kats.py counts them as `in_callback_asserts` and does
# not read them).  Each entry replaces the fixture's `expect` with what the callback body checks event by
# event; the final counter asserts of these tests count callbacks or conditional branches, so they are
# restated here in terms of the delivered events.  Keys: col_seq = the values of one column over every
# delivered event in order; col_in = every delivered value of a column lies in the set; calls = events
# per callback; create_error = createSiddhiAppRuntime throws.
LB = "LengthBatchWindowTestCase."
ONES = [1] * 9
MANUAL = {
    # :99-117 stream callback of `insert all events`: a non-expiring event's volume is the running in-count,
    # every other event from the 5th on is the expired one (volume = running remove count); 6 in, 2 removed
    "LengthWindowTestCase.lengthWindowTest2": {"rows": [], "col_seq": {"col": 2, "values": [1, 2, 3, 4, 1, 5, 2, 6]},
                                               "arrived": True},
    # :105-110 volume = running count over the 4 events of the one full batch (4 total)
    LB + "lengthBatchWindowTest2": {"rows": [], "col_seq": {"col": 2, "values": [1, 2, 3, 4]}, "arrived": True},
    # :150-169 batches of 2: each batch's current events, then (one callback later) the same events expired;
    # after every callback in - 2 == removed, which fixes the grouping to [2, 4, 4]; 6 in, 4 removed
    LB + "lengthBatchWindowTest3": {"rows": [], "col_seq": {"col": 2, "values": [1, 2, 1, 2, 3, 4, 3, 4, 5, 6]},
                                    "calls": [2, 4, 4], "arrived": True},
    # :250-256 `insert expired events`: volume = running count, 4 in total
    LB + "lengthBatchWindowTest5": {"rows": [], "col_seq": {"col": 2, "values": [1, 2, 3, 4]}, "arrived": True},
    # :500-512 lengthBatch(4, true): single-event callbacks, plus a 5-event one (4 expired + the current)
    # at each batch boundary: 7 singles, 2 five-event batches, 17 events
    LB + "lengthBatchWindowTest10": {"rows": [], "calls": [1, 1, 1, 1, 5, 1, 1, 1, 5], "arrived": True},
    # :557-571 single-event callbacks (9), count() in (0, 4]
    LB + "lengthBatchWindowTest11": {"rows": [], "calls": ONES, "col_in": {"col": 2, "values": [1, 2, 3, 4]},
                                     "arrived": True},
    # :615-627 `insert expired events` with count(): two single-event callbacks, count 0
    LB + "lengthBatchWindowTest12": {"rows": [], "calls": [1, 1], "col_in": {"col": 2, "values": [0]},
                                     "arrived": True},
    # :767-779 lengthBatch(1, true), all events: 9 single-event callbacks with count 1
    LB + "lengthBatchWindowTest15": {"rows": [], "calls": ONES, "col_in": {"col": 2, "values": [1]}, "arrived": True},
    # :823-835 lengthBatch(1): same
    LB + "lengthBatchWindowTest16": {"rows": [], "calls": ONES, "col_in": {"col": 2, "values": [1]}, "arrived": True},
    # :879-891 lengthBatch(0): 9 single-event callbacks with count 0
    LB + "lengthBatchWindowTest17": {"rows": [], "calls": ONES, "col_in": {"col": 2, "values": [0]}, "arrived": True},
    # :911 @Test(expectedExceptions = SiddhiAppCreationException): lengthBatch(1, true, 100)
    LB + "lengthBatchWindowTest18": {"rows": [], "create_error": True},
    # :997 @Test(expectedExceptions = SiddhiAppCreationException): lengthBatch(1, 1/2)
    LB + "lengthBatchWindowTest20": {"rows": [], "create_error": True},
    # @Test(expectedExceptions = SiddhiAppCreationException): parameter validation at creation
    LB + "lengthBatchWindowTest19": {"rows": [], "create_error": True},          # :967 lengthBatch(1/2)
    "LengthWindowTestCase.lengthWindowTest5": {"rows": [], "create_error": True},  # :255 length(2, price)
    "LengthWindowTestCase.sumAggregatorTest57": {"rows": [], "create_error": True},  # :283 sum(weight, deviceId)
    "LengthWindowTestCase.sumAggregatorTest58": {"rows": [], "create_error": True},
    "LengthWindowTestCase.avgAggregatorTest59": {"rows": [], "create_error": True},  # :353 avg with 2 parameters
    "TimeWindowTestCase.timeWindowTest4": {"rows": [], "create_error": True},      # :177 time(2 sec, 5)
    "TimeWindowTestCase.timeWindowTest5": {"rows": [], "create_error": True},      # :193 time(<attribute>)
    "TimeWindowTestCase.timeWindowTest6": {"rows": [], "create_error": True},      # :209 time(4.7)
    "OrderByLimitTestCase.limitTest18": {"rows": [], "create_error": True},        # :758 limit -1
    "OrderByLimitTestCase.limitTest19": {"rows": [], "create_error": True},        # :793 offset -1
    # :1069-1082 lengthBatch(3, true): 9 single-event callbacks, count() in {1, 2, 3}
    LB + "lengthBatchWindowTest21": {"rows": [], "calls": ONES, "col_in": {"col": 2, "values": [1, 2, 3]},
                                     "arrived": True},
    # :1125-1139 the same over one send(Event[]) of 9 events
    LB + "lengthBatchWindowTest22": {"rows": [], "calls": ONES, "col_in": {"col": 2, "values": [1, 2, 3]},
                                     "arrived": True},
}


def fix_inputs(k):
    """CountPatternTestCase.testQuery16 sends a long (`++now`) into the string attribute `id`, which the
    query never reads (Siddhi does not check attribute types at send): transcribed as its decimal string."""
    if k["name"] == "CountPatternTestCase.testQuery16":
        for op in k["ops"]:
            if op[0] == "send":
                op[3][0] = str(op[3][0])
    return k


def main():
    auto = json.load(open(os.path.join(HERE, "kats_auto.json")))
    for k in auto:
        if k["name"] in MANUAL:
            k["expect"] = MANUAL[k["name"]]
        fix_inputs(k)
    kept = [k for k in auto if k["name"] not in EXCLUDE]
    json.dump(kept, open(os.path.join(HERE, "kats.json"), "w"), indent=1)
    print(f"kept {len(kept)} of {len(auto)}")


if __name__ == "__main__":
    main()
