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
    "LengthWindowTestCase.lengthWindowTest5": "expects SiddhiAppCreationException",
    "LengthWindowTestCase.sumAggregatorTest57": "expects SiddhiAppCreationException (sum with 2 parameters)",
    "LengthWindowTestCase.sumAggregatorTest58": "expects SiddhiAppCreationException (sum with 2 parameters)",
    "LengthWindowTestCase.avgAggregatorTest59": "expects SiddhiAppCreationException (avg with 2 parameters)",
    "TimeWindowTestCase.timeWindowTest4": "expects SiddhiAppCreationException",
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
    "LengthBatchWindowTestCase.lengthBatchWindowTest19": "asserts SiddhiAppCreationException for lengthBatch(1/2)",
    "TimeWindowTestCase.timeWindowTest5": "asserts a creation-time validation error",
    "TimeWindowTestCase.timeWindowTest6": "asserts a creation-time validation error",
}
EXCLUDE.update({
    "OrderByLimitTestCase.limitTest18": "expects SiddhiAppCreationException (negative limit)",
    "OrderByLimitTestCase.limitTest19": "expects SiddhiAppCreationException (negative offset)",
    "GroupByTestCase.testGroupByQuery2": "timeBatch window (out of scope: SURVEY.md §2 windows row)",
    "WindowPartitionTestCase.testWindowPartitionQuery3": "scalar function default (out of scope: executor/function)",
    "WindowPartitionTestCase.testWindowPartitionQuery5": "timeBatch window (out of scope: SURVEY.md §2 windows row)",
})


def main():
    auto = json.load(open(os.path.join(HERE, "kats_auto.json")))
    kept = [k for k in auto if k["name"] not in EXCLUDE]
    json.dump(kept, open(os.path.join(HERE, "kats.json"), "w"), indent=1)
    print(f"kept {len(kept)} of {len(auto)}")


if __name__ == "__main__":
    main()
