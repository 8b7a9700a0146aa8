package io.siddhi.gpu.ext;

import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.executor.ExpressionExecutor;
import io.siddhi.core.query.processor.ProcessingMode;
import io.siddhi.core.query.selector.attribute.aggregator.AttributeAggregatorExecutor;
import io.siddhi.core.util.config.ConfigReader;
import io.siddhi.core.util.snapshot.state.State;
import io.siddhi.core.util.snapshot.state.StateFactory;
import io.siddhi.query.api.definition.Attribute;

import java.util.HashMap;
import java.util.Map;

/**
 * `sum`, `avg`, `count`, `min`, `max` backed by include/siddhi_gfx_ext.h (sg_agg_*): the native state runs
 * the built-ins' arithmetic (long sum removed through double, the min/max deque's removeFirstOccurrence,
 * canDestroy), shared with every device selector stage (siddhi_amd/csrc/selector.hpp AggOps).
 */
public final class GpuAttributeAggregators {
    private GpuAttributeAggregators() {
    }

    static int sgType(Attribute.Type t) {
        switch (t) {
            case STRING: return 0;
            case INT: return 1;
            case LONG: return 2;
            case FLOAT: return 3;
            case DOUBLE: return 4;
            case BOOL: return 5;
            default: throw new IllegalArgumentException("aggregator argument of type " + t);
        }
    }

    static Attribute.Type attrType(int sg) {
        switch (sg) {
            case 1: return Attribute.Type.INT;
            case 2: return Attribute.Type.LONG;
            case 3: return Attribute.Type.FLOAT;
            default: return Attribute.Type.DOUBLE;
        }
    }

    static long slot(Object v, int sgType) {
        switch (sgType) {
            case 3: return Float.floatToRawIntBits((Float) v) & 0xffffffffL;
            case 4: return Double.doubleToRawLongBits((Double) v);
            default: return ((Number) v).longValue();
        }
    }

    static Object value(long s, int sgType) {
        switch (sgType) {
            case 1: return (int) s;
            case 2: return s;
            case 3: return Float.intBitsToFloat((int) s);
            default: return Double.longBitsToDouble(s);
        }
    }

    /** Per group / partition state: one native aggregator. */
    static final class AggState extends State {
        final long handle;
        // written after every native call on `handle`: keeps this state reachable until the call returns, so
        // NativeHandles' phantom-reference release cannot free the handle under it (no reachabilityFence in Java 8)
        volatile int reach;

        AggState(int kind, int inType, boolean track) {
            handle = NativeExt.aggCreate(kind, inType, track);
            NativeHandles.track(this, handle, NativeExt::aggDestroy);
        }

        @Override
        public boolean canDestroy() {
            boolean r = NativeExt.aggCanDestroy(handle);
            reach = 1;
            return r;
        }

        /** The executors' state maps (e.g. SumAttributeAggregatorExecutor.AggregatorState.snapshot). */
        @Override
        public Map<String, Object> snapshot() {
            Map<String, Object> s = new HashMap<>();
            s.put("Native", NativeExt.aggSnapshot(handle));
            reach = 1;
            return s;
        }

        @Override
        public void restore(Map<String, Object> state) {
            NativeExt.aggRestore(handle, (byte[]) state.get("Native"));
            reach = 1;
        }
    }

    /** The common executor: `kind` is NativeExt.AGG_*. */
    abstract static class Base extends AttributeAggregatorExecutor<AggState> {
        private final int kind;
        private int inType;
        private int outType;
        private final byte[] isNull = new byte[1];

        Base(int kind) {
            this.kind = kind;
        }

        @Override
        protected StateFactory<AggState> init(ExpressionExecutor[] args, ProcessingMode processingMode,
                                              boolean outputExpectsExpiredEvents, ConfigReader configReader,
                                              SiddhiQueryContext siddhiQueryContext) {
            inType = args.length == 0 ? 2 : sgType(args[0].getReturnType());
            // MinAttributeAggregatorExecutor.java:95-98: trackFutureStates
            final boolean track = processingMode == ProcessingMode.SLIDE || outputExpectsExpiredEvents;
            long probe = NativeExt.aggCreate(kind, inType, track);
            outType = NativeExt.aggOutType(probe);
            NativeExt.aggDestroy(probe);
            return () -> new AggState(kind, inType, track);
        }

        private Object run(int type, Object data, AggState s) {
            boolean nul = data == null;
            long r = NativeExt.aggProcess1(s.handle, type, nul ? 0 : slot(data, inType), nul, isNull);
            s.reach = 1;
            return isNull[0] != 0 ? null : value(r, outType);
        }

        @Override
        public Object processAdd(Object data, AggState s) {
            return run(NativeExt.EV_CURRENT, data, s);
        }

        @Override
        public Object processAdd(Object[] data, AggState s) {
            return run(NativeExt.EV_CURRENT, data.length == 0 ? 0L : data[0], s);
        }

        @Override
        public Object processRemove(Object data, AggState s) {
            return run(NativeExt.EV_EXPIRED, data, s);
        }

        @Override
        public Object processRemove(Object[] data, AggState s) {
            return run(NativeExt.EV_EXPIRED, data.length == 0 ? 0L : data[0], s);
        }

        @Override
        public Object reset(AggState s) {
            return run(NativeExt.EV_RESET, null, s);
        }

        @Override
        public Attribute.Type getReturnType() {
            return attrType(outType);
        }
    }

    /** sum (SumAttributeAggregatorExecutor.java:69-355). */
    public static class Sum extends Base {
        public Sum() {
            super(NativeExt.AGG_SUM);
        }
    }

    /** avg (AvgAttributeAggregatorExecutor.java:64-390). */
    public static class Avg extends Base {
        public Avg() {
            super(NativeExt.AGG_AVG);
        }
    }

    /** count (CountAttributeAggregatorExecutor.java:67-146). */
    public static class Count extends Base {
        public Count() {
            super(NativeExt.AGG_COUNT);
        }
    }

    /** min (MinAttributeAggregatorExecutor.java:69-495). */
    public static class Min extends Base {
        public Min() {
            super(NativeExt.AGG_MIN);
        }
    }

    /** max (MaxAttributeAggregatorExecutor.java:69-475). */
    public static class Max extends Base {
        public Max() {
            super(NativeExt.AGG_MAX);
        }
    }
}
