package io.siddhi.gpu.ext;

import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.event.ComplexEvent;
import io.siddhi.core.event.ComplexEventChunk;
import io.siddhi.core.event.state.StateEvent;
import io.siddhi.core.event.stream.StreamEvent;
import io.siddhi.core.event.stream.StreamEventCloner;
import io.siddhi.core.executor.ConstantExpressionExecutor;
import io.siddhi.core.executor.ExpressionExecutor;
import io.siddhi.core.executor.VariableExpressionExecutor;
import io.siddhi.core.query.processor.Processor;
import io.siddhi.core.query.processor.SchedulingProcessor;
import io.siddhi.core.query.processor.stream.window.BatchWindowProcessor;
import io.siddhi.core.query.processor.stream.window.SlidingFindableWindowProcessor;
import io.siddhi.core.table.Table;
import io.siddhi.core.util.Scheduler;
import io.siddhi.core.util.collection.operator.CompiledCondition;
import io.siddhi.core.util.collection.operator.MatchingMetaInfoHolder;
import io.siddhi.core.util.config.ConfigReader;
import io.siddhi.core.util.parser.OperatorParser;
import io.siddhi.core.util.snapshot.state.StateFactory;
import io.siddhi.query.api.exception.SiddhiAppValidationException;
import io.siddhi.query.api.expression.Expression;

import java.util.List;
import java.util.Map;

/**
 * `length`, `time` and `lengthBatch` backed by include/siddhi_gfx_ext.h (sg_window_*), registered with
 * SiddhiManager.setExtension by {@link GpuExtensions}.  Parameter handling follows the replaced built-ins
 * (LengthWindowProcessor.init, TimeWindowProcessor.init, LengthBatchWindowProcessor.init); the queue
 * discipline runs natively (siddhi_amd/csrc/window_proc.hpp), so the output chunks and their order are the
 * built-ins'.  Findable windows answer joins / `find` over the clones they hold, as the built-ins do.
 */
public final class GpuWindowProcessors {
    private GpuWindowProcessors() {
    }

    static long constant(ExpressionExecutor e, String what) {
        if (!(e instanceof ConstantExpressionExecutor)) {
            throw new SiddhiAppValidationException(what + " must be a constant");
        }
        Object v = ((ConstantExpressionExecutor) e).getValue();
        return v instanceof Integer ? (Integer) v : (Long) v;
    }

    static long now(SiddhiQueryContext q) {
        return q.getSiddhiAppContext().getTimestampGenerator().currentTime();
    }

    /** #window.length(L) (LengthWindowProcessor.java:106-141). */
    public static class Length extends SlidingFindableWindowProcessor<GpuWindowState> {
        private long length;

        @Override
        protected StateFactory<GpuWindowState> init(ExpressionExecutor[] args, ConfigReader configReader,
                                                    SiddhiQueryContext siddhiQueryContext) {
            if (args.length != 1) {
                throw new SiddhiAppValidationException("Length window should only have one parameter (<int> "
                        + "window.length), but found " + args.length + " input parameters.");
            }
            length = constant(args[0], "window.length");
            return () -> new GpuWindowState(NativeExt.WIN_LENGTH, length, false, true);
        }

        @Override
        protected void process(ComplexEventChunk<StreamEvent> chunk, Processor next, StreamEventCloner cloner,
                               GpuWindowState state) {
            List<ComplexEventChunk<StreamEvent>> out;
            synchronized (state) {
                out = state.process(chunk, cloner, now(siddhiQueryContext));
            }
            for (ComplexEventChunk<StreamEvent> c : out) {
                next.process(c);
            }
        }

        @Override
        public CompiledCondition compileCondition(Expression condition, MatchingMetaInfoHolder holder,
                                                  List<VariableExpressionExecutor> vars, Map<String, Table> tables,
                                                  GpuWindowState state, SiddhiQueryContext ctx) {
            return OperatorParser.constructOperator(state.held.values(), condition, holder, vars, tables, ctx);
        }

        @Override
        public StreamEvent find(StateEvent matchingEvent, CompiledCondition compiledCondition,
                                StreamEventCloner cloner, GpuWindowState state) {
            return ((io.siddhi.core.util.collection.operator.Operator) compiledCondition)
                    .find(matchingEvent, state.held.values(), cloner);
        }

        @Override
        public void start() {
        }

        @Override
        public void stop() {
        }
    }

    /** #window.time(T) (TimeWindowProcessor.java:133-169) with its Scheduler (notifyAt per new timestamp). */
    public static class Time extends SlidingFindableWindowProcessor<GpuWindowState> implements SchedulingProcessor {
        private long timeInMillis;
        private Scheduler scheduler;

        @Override
        protected StateFactory<GpuWindowState> init(ExpressionExecutor[] args, ConfigReader configReader,
                                                    SiddhiQueryContext siddhiQueryContext) {
            if (args.length != 1) {
                throw new SiddhiAppValidationException("Time window should only have one parameter (<int|long|time> "
                        + "window.time), but found " + args.length + " input parameters.");
            }
            timeInMillis = constant(args[0], "window.time");
            return () -> new GpuWindowState(NativeExt.WIN_TIME, timeInMillis, false, true);
        }

        @Override
        public void setScheduler(Scheduler scheduler) {
            this.scheduler = scheduler;
        }

        @Override
        public Scheduler getScheduler() {
            return scheduler;
        }

        @Override
        protected void process(ComplexEventChunk<StreamEvent> chunk, Processor next, StreamEventCloner cloner,
                               GpuWindowState state) {
            List<ComplexEventChunk<StreamEvent>> out;
            synchronized (state) {
                boolean timer = false;
                chunk.reset();
                while (chunk.hasNext()) {
                    timer |= chunk.next().getType() == ComplexEvent.Type.TIMER;
                }
                long now = now(siddhiQueryContext);
                out = timer ? state.onTime(now, cloner) : state.process(chunk, cloner, now);
                // TimeWindowProcessor.java:158-160: notifyAt(ts + T) once per new timestamp -- every deadline
                // the native window queued in this call, in order (not only a changed front)
                for (long d : state.takeDeadlines()) {
                    scheduler.notifyAt(d);
                }
            }
            for (ComplexEventChunk<StreamEvent> c : out) {
                next.process(c);
            }
        }

        @Override
        public CompiledCondition compileCondition(Expression condition, MatchingMetaInfoHolder holder,
                                                  List<VariableExpressionExecutor> vars, Map<String, Table> tables,
                                                  GpuWindowState state, SiddhiQueryContext ctx) {
            return OperatorParser.constructOperator(state.held.values(), condition, holder, vars, tables, ctx);
        }

        @Override
        public StreamEvent find(StateEvent matchingEvent, CompiledCondition compiledCondition,
                                StreamEventCloner cloner, GpuWindowState state) {
            return ((io.siddhi.core.util.collection.operator.Operator) compiledCondition)
                    .find(matchingEvent, state.held.values(), cloner);
        }

        @Override
        public void start() {
        }

        @Override
        public void stop() {
        }
    }

    /** #window.lengthBatch(L[, streamCurrentEvents]) (LengthBatchWindowProcessor.java:154-351). */
    public static class LengthBatch extends BatchWindowProcessor<GpuWindowState> {
        private long length;
        private boolean streamCurrent;

        @Override
        protected StateFactory<GpuWindowState> init(ExpressionExecutor[] args, ConfigReader configReader,
                                                    boolean outputExpectsExpiredEvents,
                                                    SiddhiQueryContext siddhiQueryContext) {
            if (args.length < 1 || args.length > 2) {
                throw new SiddhiAppValidationException("LengthBatch window should have one or two parameters "
                        + "(<int> window.length, <bool> stream.current.event), but found " + args.length);
            }
            length = constant(args[0], "window.length");
            streamCurrent = args.length == 2
                    && (Boolean) ((ConstantExpressionExecutor) args[1]).getValue();
            final boolean expiredOn = outputExpectsExpiredEvents;
            return () -> new GpuWindowState(NativeExt.WIN_LENGTH_BATCH, length, streamCurrent, expiredOn);
        }

        @Override
        protected void process(ComplexEventChunk<StreamEvent> chunk, Processor next, StreamEventCloner cloner,
                               GpuWindowState state) {
            List<ComplexEventChunk<StreamEvent>> out;
            synchronized (state) {
                out = state.process(chunk, cloner, now(siddhiQueryContext));
            }
            for (ComplexEventChunk<StreamEvent> c : out) {
                next.process(c);
            }
        }

        @Override
        public void start() {
        }

        @Override
        public void stop() {
        }
    }
}
