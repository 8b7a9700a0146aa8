package io.siddhi.gpu;

import io.siddhi.query.api.SiddhiApp;
import io.siddhi.query.api.annotation.Annotation;
import io.siddhi.query.api.annotation.Element;
import io.siddhi.query.api.definition.Attribute;
import io.siddhi.query.api.definition.StreamDefinition;
import io.siddhi.query.api.execution.ExecutionElement;
import io.siddhi.query.api.execution.partition.Partition;
import io.siddhi.query.api.execution.partition.PartitionType;
import io.siddhi.query.api.execution.partition.ValuePartitionType;
import io.siddhi.query.api.execution.query.Query;
import io.siddhi.query.api.execution.query.input.handler.Filter;
import io.siddhi.query.api.execution.query.input.handler.StreamHandler;
import io.siddhi.query.api.execution.query.input.handler.Window;
import io.siddhi.query.api.execution.query.input.state.AbsentStreamStateElement;
import io.siddhi.query.api.execution.query.input.state.CountStateElement;
import io.siddhi.query.api.execution.query.input.state.EveryStateElement;
import io.siddhi.query.api.execution.query.input.state.LogicalStateElement;
import io.siddhi.query.api.execution.query.input.state.NextStateElement;
import io.siddhi.query.api.execution.query.input.state.StateElement;
import io.siddhi.query.api.execution.query.input.state.StreamStateElement;
import io.siddhi.query.api.execution.query.input.stream.InputStream;
import io.siddhi.query.api.execution.query.input.stream.SingleInputStream;
import io.siddhi.query.api.execution.query.input.stream.StateInputStream;
import io.siddhi.query.api.execution.query.output.stream.InsertIntoStream;
import io.siddhi.query.api.execution.query.output.stream.OutputStream;
import io.siddhi.query.api.execution.query.selection.OrderByAttribute;
import io.siddhi.query.api.execution.query.selection.OutputAttribute;
import io.siddhi.query.api.execution.query.selection.Selector;
import io.siddhi.query.api.expression.AttributeFunction;
import io.siddhi.query.api.expression.Expression;
import io.siddhi.query.api.expression.Variable;
import io.siddhi.query.api.expression.condition.And;
import io.siddhi.query.api.expression.condition.Compare;
import io.siddhi.query.api.expression.condition.IsNull;
import io.siddhi.query.api.expression.condition.Not;
import io.siddhi.query.api.expression.condition.Or;
import io.siddhi.query.api.expression.constant.BoolConstant;
import io.siddhi.query.api.expression.constant.Constant;
import io.siddhi.query.api.expression.constant.DoubleConstant;
import io.siddhi.query.api.expression.constant.FloatConstant;
import io.siddhi.query.api.expression.constant.IntConstant;
import io.siddhi.query.api.expression.constant.LongConstant;
import io.siddhi.query.api.expression.constant.StringConstant;
import io.siddhi.query.api.expression.math.Add;
import io.siddhi.query.api.expression.math.Divide;
import io.siddhi.query.api.expression.math.ModExpression;
import io.siddhi.query.api.expression.math.Multiply;
import io.siddhi.query.api.expression.math.Subtract;

import java.util.ArrayList;
import java.util.IdentityHashMap;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

/**
 * Emits the version-1 app descriptor (include/siddhi_gfx_descriptor.schema.json) from a parsed
 * {@link SiddhiApp}: the Java twin of siddhi_amd/ql.py's resolution step, so the device runtime is driven
 * without the Python front end.
 *
 * <ul>
 * <li>MetaStateEvent slot order = the order StateInputStreamParser.parse visits the stream elements
 *     (next: current then next; logical: element 2 then element 1; StateInputStreamParser.java:148-408).</li>
 * <li>Variables resolve as ExpressionParser.parseVariable does (ExpressionParser.java:1255-1440): a
 *     reference names a slot; the chain index is the variable's stream index ([0], [last] = -2, [last-k]),
 *     filters of a count state default to the current (last) event, selector variables to index 0; an
 *     unindexed reference to a count state in the selector is a multi-value variable.</li>
 * <li>Result types follow Java binary numeric promotion as Siddhi's executor factories apply it;
 *     aggregator output types are those of Sum/Avg/Count/Min/MaxAttributeAggregatorExecutor.</li>
 * </ul>
 * Execution elements are emitted in app order (queries and partition bodies interleaved), which is the
 * order SiddhiAppRuntimeBuilder subscribes the queries to their junctions.
 */
public final class DescriptorEmitter {
    private final SiddhiApp app;
    private final Map<String, List<Attribute>> streams = new LinkedHashMap<>();
    /** per emitted query: output attribute types, and the input streams it reads */
    final Map<String, Attribute.Type[]> queryOutTypes = new LinkedHashMap<>();
    final Map<String, List<Attribute>> queryOutAttrs = new LinkedHashMap<>();   // selector output attributes
    final Map<String, String> queryOutStream = new LinkedHashMap<>();           // `insert into` target (no '#')
    final Map<String, List<String>> queryInputs = new LinkedHashMap<>();

    public DescriptorEmitter(SiddhiApp app) {
        this.app = app;
        for (StreamDefinition d : app.getStreamDefinitionMap().values()) {
            streams.put(d.getId(), d.getAttributeList());
        }
    }

    /** The descriptor JSON of the whole app. */
    public String emit() {
        List<String> queries = new ArrayList<>();
        int anon = 0;
        for (ExecutionElement ee : app.getExecutionElementList()) {
            if (ee instanceof Query) {
                queries.add(query((Query) ee, null, "query" + (++anon)));
            } else if (ee instanceof Partition) {
                Partition p = (Partition) ee;
                partitionId++;
                purge = purgeOf(p);
                Map<String, Integer> keyed = new LinkedHashMap<>();
                for (Map.Entry<String, PartitionType> e : p.getPartitionTypeMap().entrySet()) {
                    if (!(e.getValue() instanceof ValuePartitionType)) {
                        throw new UnsupportedOnGpuException("range partitions are not lowered");
                    }
                    Expression k = ((ValuePartitionType) e.getValue()).getExpression();
                    if (!(k instanceof Variable)) {
                        throw new UnsupportedOnGpuException("partition key is not an attribute");
                    }
                    keyed.put(e.getKey(), attrIndex(e.getKey(), ((Variable) k).getAttributeName()));
                }
                for (Query q : p.getQueryList()) {
                    queries.add(query(q, keyed, "query" + (++anon)));
                }
            }
        }
        StringBuilder s = new StringBuilder("{\"version\":1,\"name\":").append(str(app.getName()));
        s.append(",\"playback\":").append(playback());
        s.append(",\"streams\":{");
        boolean first = true;
        for (Map.Entry<String, List<Attribute>> e : streams.entrySet()) {
            if (!first) {
                s.append(',');
            }
            first = false;
            s.append(str(e.getKey())).append(":[");
            for (int i = 0; i < e.getValue().size(); i++) {
                Attribute a = e.getValue().get(i);
                s.append(i > 0 ? "," : "").append('[').append(str(a.getName())).append(',')
                        .append(str(a.getType().name())).append(']');
            }
            s.append(']');
        }
        s.append("},\"queries\":[").append(String.join(",", queries)).append("]}");
        return s.toString();
    }

    /** The attribute list of a defined (or insert-into-defined) stream. */
    List<Attribute> streamAttributes(String stream) {
        return streams.get(stream);
    }

    Map<String, List<Attribute>> allStreams() {
        return streams;
    }

    private boolean playback() {
        for (Annotation a : app.getAnnotations()) {
            if (a.getName().equalsIgnoreCase("app:playback") || a.getName().equalsIgnoreCase("playback")) {
                return true;
            }
        }
        return false;
    }

    // ---- one query ----------------------------------------------------------------------------

    /** (stream, reference, multi) of one MetaStateEvent position. */
    private static final class Slot {
        final String stream;
        final String ref;
        final boolean multi;

        Slot(String stream, String ref, boolean multi) {
            this.stream = stream;
            this.ref = ref;
            this.multi = multi;
        }
    }

    private List<Slot> slots;
    private boolean single;
    private List<String[]> outAttrs;

    private int partitionId = -1;
    private String purge;   // the current partition block's @purge as descriptor JSON, or null

    /** PartitionRuntimeImpl constructor (:120-147): @purge(enable, idle.period[, interval]). */
    private static String purgeOf(Partition p) {
        for (Annotation a : p.getAnnotations()) {
            if (!a.getName().equalsIgnoreCase("purge")) {
                continue;
            }
            String enable = a.getElement("enable");
            String idle = a.getElement("idle.period");
            String interval = a.getElement("interval");
            if (enable == null || idle == null) {
                throw new UnsupportedOnGpuException("@purge needs 'enable' and 'idle.period'");
            }
            if (!Boolean.parseBoolean(enable)) {
                return null;
            }
            long iv = interval == null ? 300000L : Expression.Time.timeToLong(interval);
            return "{\"interval\":" + iv + ",\"idle\":" + Expression.Time.timeToLong(idle) + "}";
        }
        return null;
    }

    private String query(Query q, Map<String, Integer> partition, String fallbackName) {
        String name = fallbackName;
        for (Annotation a : q.getAnnotations()) {
            if (a.getName().equalsIgnoreCase("info")) {
                for (Element el : a.getElements()) {
                    if ("name".equalsIgnoreCase(el.getKey())) {
                        name = el.getValue();
                    }
                }
            }
        }
        InputStream in = q.getInputStream();
        String input;
        outAttrs = new ArrayList<>();
        if (in instanceof SingleInputStream) {
            SingleInputStream si = (SingleInputStream) in;
            single = true;
            slots = new ArrayList<>();
            slots.add(new Slot(si.getStreamId(), si.getStreamReferenceId(), false));
            StringBuilder h = new StringBuilder();
            for (StreamHandler sh : si.getStreamHandlers()) {
                if (h.length() > 0) {
                    h.append(',');
                }
                if (sh instanceof Filter) {
                    h.append("{\"k\":\"filter\",\"e\":").append(expr(((Filter) sh).getParameters()[0], -1, -1, false,
                            false)).append('}');
                } else if (sh instanceof Window) {
                    Window w = (Window) sh;
                    List<String> ps = new ArrayList<>();
                    for (Expression p : w.getParameters()) {
                        ps.add(expr(p, -1, -1, false, false));
                    }
                    h.append("{\"k\":\"window\",\"name\":").append(str(w.getName())).append(",\"params\":[")
                            .append(String.join(",", ps)).append("]}");
                } else {
                    throw new UnsupportedOnGpuException("stream function " + sh);
                }
            }
            input = "{\"kind\":\"single\",\"stream\":" + str(si.getStreamId()) + ",\"handlers\":[" + h + "]}";
        } else if (in instanceof StateInputStream) {
            StateInputStream st = (StateInputStream) in;
            single = false;
            List<StreamStateElement> order = new ArrayList<>();
            Map<StreamStateElement, Boolean> multi = new IdentityHashMap<>();
            slotOrder(st.getStateElement(), order, multi, false);
            slots = new ArrayList<>();
            Map<StreamStateElement, Integer> slotOf = new IdentityHashMap<>();
            for (StreamStateElement e : order) {
                slotOf.put(e, slots.size());
                SingleInputStream b = e.getBasicSingleInputStream();
                slots.add(new Slot(b.getStreamId(), b.getStreamReferenceId(), multi.containsKey(e)));
            }
            StringBuilder sl = new StringBuilder();
            for (Slot s : slots) {
                sl.append(sl.length() > 0 ? "," : "").append("{\"stream\":").append(str(s.stream)).append(",\"ref\":")
                        .append(s.ref == null ? "null" : str(s.ref)).append(",\"multi\":").append(s.multi).append('}');
            }
            input = "{\"kind\":\"state\",\"type\":" + str(st.getStateType().name()) + ",\"within\":"
                    + (st.getWithinTime() == null ? "null" : st.getWithinTime().value()) + ",\"element\":"
                    + element(st.getStateElement(), slotOf) + ",\"slots\":[" + sl + "]}";
        } else {
            throw new UnsupportedOnGpuException("join / other input streams are not lowered");
        }
        String select = selector(q.getSelector());
        OutputStream os = q.getOutputStream();
        String events;
        switch (os.getOutputEventType()) {
            case EXPIRED_EVENTS:
                events = "expired";
                break;
            case ALL_EVENTS:
                events = "all";
                break;
            default:
                events = "current";
        }
        String output = os instanceof InsertIntoStream
                ? "{\"kind\":\"insert\",\"stream\":" + str(os.getId()) + ",\"events\":\"" + events + "\"}"
                : "{\"kind\":\"return\",\"events\":\"" + events + "\"}";
        if (os instanceof InsertIntoStream && !streams.containsKey(os.getId())) {
            // SiddhiAppParser defines an undefined insert-into target from the selector's output attributes
            List<Attribute> as = new ArrayList<>();
            for (String[] a : outAttrs) {
                as.add(new Attribute(a[0], Attribute.Type.valueOf(a[1])));
            }
            streams.put(os.getId(), as);
        }
        Attribute.Type[] ot = new Attribute.Type[outAttrs.size()];
        for (int i = 0; i < ot.length; i++) {
            ot[i] = Attribute.Type.valueOf(outAttrs.get(i)[1]);
        }
        queryOutTypes.put(name, ot);
        List<Attribute> oas = new ArrayList<>();
        for (String[] a : outAttrs) {
            oas.add(new Attribute(a[0], Attribute.Type.valueOf(a[1])));
        }
        queryOutAttrs.put(name, oas);
        if (os instanceof InsertIntoStream && !((InsertIntoStream) os).isInnerStream()) {
            queryOutStream.put(name, os.getId());
        }
        List<String> ins = new ArrayList<>();
        for (Slot s : slots) {
            if (!ins.contains(s.stream)) {
                ins.add(s.stream);
            }
        }
        queryInputs.put(name, ins);
        StringBuilder oa = new StringBuilder();
        for (String[] a : outAttrs) {
            oa.append(oa.length() > 0 ? "," : "").append('[').append(str(a[0])).append(',').append(str(a[1])).append(']');
        }
        StringBuilder d = new StringBuilder("{\"name\":").append(str(name)).append(",\"input\":").append(input)
                .append(",\"select\":").append(select).append(",\"output\":").append(output)
                .append(",\"out_attrs\":[").append(oa).append(']');
        if (partition != null) {
            d.append(",\"partition\":{");
            boolean first = true;
            for (Map.Entry<String, Integer> e : partition.entrySet()) {
                d.append(first ? "" : ",").append(str(e.getKey())).append(':').append(e.getValue());
                first = false;
            }
            d.append('}');
            d.append(",\"partition_id\":").append(partitionId);
            if (purge != null) {
                d.append(",\"purge\":").append(purge);
            }
        }
        return d.append('}').toString();
    }

    private void slotOrder(StateElement el, List<StreamStateElement> out, Map<StreamStateElement, Boolean> multi,
                           boolean inCount) {
        if (el instanceof StreamStateElement) {     // includes AbsentStreamStateElement
            out.add((StreamStateElement) el);
            if (inCount) {
                multi.put((StreamStateElement) el, true);
            }
        } else if (el instanceof NextStateElement) {
            slotOrder(((NextStateElement) el).getStateElement(), out, multi, false);
            slotOrder(((NextStateElement) el).getNextStateElement(), out, multi, false);
        } else if (el instanceof EveryStateElement) {
            slotOrder(((EveryStateElement) el).getStateElement(), out, multi, false);
        } else if (el instanceof LogicalStateElement) {
            slotOrder(((LogicalStateElement) el).getStreamStateElement2(), out, multi, false);
            slotOrder(((LogicalStateElement) el).getStreamStateElement1(), out, multi, false);
        } else if (el instanceof CountStateElement) {
            slotOrder(((CountStateElement) el).getStreamStateElement(), out, multi, true);
        }
    }

    private String element(StateElement el, Map<StreamStateElement, Integer> slotOf) {
        if (el instanceof StreamStateElement) {
            StreamStateElement s = (StreamStateElement) el;
            int slot = slotOf.get(s);
            List<String> fs = new ArrayList<>();
            for (StreamHandler h : s.getBasicSingleInputStream().getStreamHandlers()) {
                if (!(h instanceof Filter)) {
                    throw new UnsupportedOnGpuException("stream handler inside a state element");
                }
                fs.add(expr(((Filter) h).getParameters()[0], slot, -1, false, false));
            }
            StringBuilder b = new StringBuilder("{\"k\":");
            if (el instanceof AbsentStreamStateElement) {
                AbsentStreamStateElement a = (AbsentStreamStateElement) el;
                b.append("\"absent\",\"wait\":").append(a.getWaitingTime() == null ? "null" : a.getWaitingTime().value());
            } else {
                b.append("\"stream\"");
            }
            return b.append(",\"stream\":").append(str(s.getBasicSingleInputStream().getStreamId())).append(",\"slot\":")
                    .append(slot).append(",\"filters\":[").append(String.join(",", fs)).append("]}").toString();
        }
        if (el instanceof NextStateElement) {
            NextStateElement n = (NextStateElement) el;
            return "{\"k\":\"next\",\"a\":" + element(n.getStateElement(), slotOf) + ",\"b\":"
                    + element(n.getNextStateElement(), slotOf) + "}";
        }
        if (el instanceof EveryStateElement) {
            return "{\"k\":\"every\",\"e\":" + element(((EveryStateElement) el).getStateElement(), slotOf) + "}";
        }
        if (el instanceof LogicalStateElement) {
            LogicalStateElement l = (LogicalStateElement) el;
            return "{\"k\":\"logical\",\"op\":" + str(l.getType().name()) + ",\"a\":"
                    + element(l.getStreamStateElement1(), slotOf) + ",\"b\":" + element(l.getStreamStateElement2(), slotOf)
                    + "}";
        }
        if (el instanceof CountStateElement) {
            CountStateElement c = (CountStateElement) el;
            return "{\"k\":\"count\",\"min\":" + c.getMinCount() + ",\"max\":" + c.getMaxCount() + ",\"e\":"
                    + element(c.getStreamStateElement(), slotOf) + "}";
        }
        throw new UnsupportedOnGpuException("state element " + el);
    }

    private String selector(Selector s) {
        List<String> attrs = new ArrayList<>();
        if (s.getSelectionList().isEmpty()) {                  // select *
            for (int si = 0; si < slots.size(); si++) {
                List<Attribute> as = streams.get(slots.get(si).stream);
                for (int i = 0; i < as.size(); i++) {
                    String t = as.get(i).getType().name();
                    attrs.add("{\"name\":" + str(as.get(i).getName()) + ",\"e\":{\"op\":\"var\",\"slot\":"
                            + (single ? -1 : si) + ",\"chain\":0,\"attr\":" + i + ",\"t\":\"" + t + "\"}}");
                    outAttrs.add(new String[]{as.get(i).getName(), t});
                }
            }
        } else {
            for (OutputAttribute oa : s.getSelectionList()) {
                String e = expr(oa.getExpression(), null, 0, false, true);
                attrs.add("{\"name\":" + str(oa.getRename()) + ",\"e\":" + e + "}");
                outAttrs.add(new String[]{oa.getRename(), lastType});
            }
        }
        List<String> gb = new ArrayList<>();
        for (Variable v : s.getGroupByList()) {
            gb.add(expr(v, null, 0, false, false));
        }
        String having = s.getHavingExpression() == null ? "null" : expr(s.getHavingExpression(), null, 0, true, true);
        List<String> ob = new ArrayList<>();
        for (OrderByAttribute o : s.getOrderByList()) {
            ob.add("[" + expr(o.getVariable(), null, 0, true, false) + ","
                    + (o.getOrder() == OrderByAttribute.Order.DESC ? "\"desc\"" : "\"asc\"") + "]");
        }
        return "{\"attrs\":[" + String.join(",", attrs) + "],\"group_by\":[" + String.join(",", gb) + "],\"having\":"
                + having + ",\"order_by\":[" + String.join(",", ob) + "],\"limit\":" + constNumber(s.getLimit())
                + ",\"offset\":" + constNumber(s.getOffset()) + "}";
    }

    // ---- expressions ---------------------------------------------------------------------------

    private String lastType;    // result type of the last expr() call

    private static final String[] RANK = {"INT", "LONG", "FLOAT", "DOUBLE"};

    private static int rank(String t) {
        for (int i = 0; i < RANK.length; i++) {
            if (RANK[i].equals(t)) {
                return i;
            }
        }
        throw new UnsupportedOnGpuException("arithmetic on " + t);
    }

    private static String promote(String a, String b) {
        return rank(a) >= rank(b) ? a : b;
    }

    private String expr(Expression e, Integer currentState, int defaultIndex, boolean having, boolean allowAgg) {
        String r;
        if (e instanceof Constant) {
            r = constant((Constant) e);
        } else if (e instanceof Variable) {
            r = variable((Variable) e, currentState, defaultIndex, having);
        } else if (e instanceof And || e instanceof Or) {
            Expression l = e instanceof And ? ((And) e).getLeftExpression() : ((Or) e).getLeftExpression();
            Expression rr = e instanceof And ? ((And) e).getRightExpression() : ((Or) e).getRightExpression();
            r = "{\"op\":\"" + (e instanceof And ? "and" : "or") + "\",\"a\":" + expr(l, currentState, defaultIndex, having,
                    allowAgg) + ",\"b\":" + expr(rr, currentState, defaultIndex, having, allowAgg) + ",\"t\":\"BOOL\"}";
            lastType = "BOOL";
        } else if (e instanceof Not) {
            r = "{\"op\":\"not\",\"a\":" + expr(((Not) e).getExpression(), currentState, defaultIndex, having, allowAgg)
                    + ",\"t\":\"BOOL\"}";
            lastType = "BOOL";
        } else if (e instanceof IsNull) {
            r = "{\"op\":\"isnull\",\"a\":" + expr(((IsNull) e).getExpression(), currentState, defaultIndex, having,
                    allowAgg) + ",\"t\":\"BOOL\"}";
            lastType = "BOOL";
        } else if (e instanceof Compare) {
            Compare c = (Compare) e;
            String a = expr(c.getLeftExpression(), currentState, defaultIndex, having, allowAgg);
            String ta = lastType;
            String b = expr(c.getRightExpression(), currentState, defaultIndex, having, allowAgg);
            String tb = lastType;
            String op;
            switch (c.getOperator()) {
                case LESS_THAN: op = "<"; break;
                case GREATER_THAN: op = ">"; break;
                case LESS_THAN_EQUAL: op = "<="; break;
                case GREATER_THAN_EQUAL: op = ">="; break;
                case EQUAL: op = "=="; break;
                default: op = "!=";
            }
            String ct;
            boolean eq = op.equals("==") || op.equals("!=");
            if (eq && (ta.equals("STRING") || ta.equals("BOOL") || tb.equals("STRING") || tb.equals("BOOL"))) {
                if (!ta.equals(tb) && !ta.equals("OBJECT") && !tb.equals("OBJECT")) {
                    throw new UnsupportedOnGpuException("cannot compare " + ta + " with " + tb);
                }
                ct = ta.equals("OBJECT") ? tb : ta;
            } else if (ta.equals("OBJECT") || tb.equals("OBJECT")) {
                ct = "OBJECT";
            } else {
                ct = promote(ta, tb);
            }
            r = "{\"op\":\"" + op + "\",\"a\":" + a + ",\"b\":" + b + ",\"ct\":\"" + ct + "\",\"t\":\"BOOL\"}";
            lastType = "BOOL";
        } else if (e instanceof Add || e instanceof Subtract || e instanceof Multiply || e instanceof Divide
                || e instanceof ModExpression) {
            Expression l;
            Expression rr;
            String op;
            if (e instanceof Add) { l = ((Add) e).getLeftValue(); rr = ((Add) e).getRightValue(); op = "+"; }
            else if (e instanceof Subtract) { l = ((Subtract) e).getLeftValue(); rr = ((Subtract) e).getRightValue(); op = "-"; }
            else if (e instanceof Multiply) { l = ((Multiply) e).getLeftValue(); rr = ((Multiply) e).getRightValue(); op = "*"; }
            else if (e instanceof Divide) { l = ((Divide) e).getLeftValue(); rr = ((Divide) e).getRightValue(); op = "/"; }
            else { l = ((ModExpression) e).getLeftValue(); rr = ((ModExpression) e).getRightValue(); op = "%"; }
            String a = expr(l, currentState, defaultIndex, having, allowAgg);
            String ta = lastType;
            String b = expr(rr, currentState, defaultIndex, having, allowAgg);
            String t = promote(ta, lastType);
            r = "{\"op\":\"" + op + "\",\"a\":" + a + ",\"b\":" + b + ",\"t\":\"" + t + "\"}";
            lastType = t;
        } else if (e instanceof AttributeFunction) {
            AttributeFunction f = (AttributeFunction) e;
            String name = f.getName().toLowerCase();
            if (!allowAgg || f.getNamespace() != null && !f.getNamespace().isEmpty()) {
                throw new UnsupportedOnGpuException("function " + f.getName() + " is not lowered");
            }
            List<String> args = new ArrayList<>();
            String at = "OBJECT";
            for (Expression p : f.getParameters()) {
                args.add(expr(p, currentState, defaultIndex, having, false));
                at = lastType;
            }
            String t;
            switch (name) {
                case "count": case "distinctcount": t = "LONG"; break;
                case "avg": case "stddev": t = "DOUBLE"; break;
                case "sum": t = at.equals("INT") || at.equals("LONG") ? "LONG" : "DOUBLE"; break;
                case "min": case "max": case "minforever": case "maxforever": t = at; break;
                default: throw new UnsupportedOnGpuException("function " + f.getName() + " is not lowered");
            }
            r = "{\"op\":\"agg\",\"name\":\"" + name + "\",\"args\":[" + String.join(",", args) + "],\"t\":\"" + t + "\"}";
            lastType = t;
        } else {
            throw new UnsupportedOnGpuException("expression " + e);
        }
        return r;
    }

    private String constant(Constant c) {
        String t;
        String v;
        if (c instanceof IntConstant) { t = "INT"; v = String.valueOf(((IntConstant) c).getValue()); }
        else if (c instanceof LongConstant) { t = "LONG"; v = String.valueOf(((LongConstant) c).getValue()); }
        else if (c instanceof FloatConstant) { t = "FLOAT"; v = Float.toString(((FloatConstant) c).getValue()); }
        else if (c instanceof DoubleConstant) { t = "DOUBLE"; v = Double.toString(((DoubleConstant) c).getValue()); }
        else if (c instanceof BoolConstant) { t = "BOOL"; v = String.valueOf(((BoolConstant) c).getValue()); }
        else if (c instanceof StringConstant) { t = "STRING"; v = str(((StringConstant) c).getValue()); }
        else { t = "OBJECT"; v = "null"; }
        lastType = t;
        return "{\"op\":\"const\",\"t\":\"" + t + "\",\"v\":" + v + "}";
    }

    private static String constNumber(Constant c) {
        if (c == null) {
            return "null";
        }
        if (c instanceof IntConstant) {
            return String.valueOf(((IntConstant) c).getValue());
        }
        if (c instanceof LongConstant) {
            return String.valueOf(((LongConstant) c).getValue());
        }
        throw new UnsupportedOnGpuException("limit / offset is not an integer");
    }

    private String variable(Variable v, Integer currentState, int defaultIndex, boolean having) {
        String ref = v.getStreamId();
        String attr = v.getAttributeName();
        if (having && ref == null) {                       // ExpressionParser.java:1316-1323
            for (int i = 0; i < outAttrs.size(); i++) {
                if (outAttrs.get(i)[0].equals(attr)) {
                    lastType = outAttrs.get(i)[1];
                    return "{\"op\":\"outvar\",\"attr\":" + i + ",\"t\":\"" + lastType + "\"}";
                }
            }
        }
        if (single) {
            Slot s = slots.get(0);
            int ai = attrIndex(s.stream, attr);
            lastType = streams.get(s.stream).get(ai).getType().name();
            return "{\"op\":\"var\",\"slot\":-1,\"chain\":0,\"attr\":" + ai + ",\"t\":\"" + lastType + "\"}";
        }
        Integer idx = v.getStreamIndex();             // null, k >= 0, or LAST (-2) - k
        int chain = idx == null ? defaultIndex : (idx <= Variable.LAST ? idx + 1 : idx);
        int slot = -1;
        boolean multi = false;
        if (ref == null) {
            if (currentState != null && currentState >= 0) {
                slot = currentState;
            } else {
                for (int i = 0; i < slots.size(); i++) {
                    if (hasAttr(slots.get(i).stream, attr)) {
                        if (slot >= 0) {
                            throw new UnsupportedOnGpuException("attribute '" + attr + "' is ambiguous");
                        }
                        slot = i;
                    }
                }
            }
        } else {
            for (int i = 0; i < slots.size(); i++) {
                Slot s = slots.get(i);
                if ((s.ref == null && s.stream.equals(ref)) || (s.ref != null && s.ref.equals(ref))) {
                    slot = i;
                    if (currentState != null && currentState > -1 && slots.get(currentState).ref != null
                            && idx != null && idx <= Variable.LAST) {
                        if (ref.equals(slots.get(currentState).ref)) {
                            chain = idx;                   // own-state [last] keeps the raw index
                        }
                    } else if (currentState == null && idx == null) {
                        multi = s.multi;
                    }
                    break;
                }
            }
        }
        if (slot < 0) {
            throw new UnsupportedOnGpuException("no stream reference for attribute '" + attr + "'");
        }
        int ai = attrIndex(slots.get(slot).stream, attr);
        lastType = streams.get(slots.get(slot).stream).get(ai).getType().name();
        if (multi) {
            lastType = "OBJECT";
            return "{\"op\":\"multivar\",\"slot\":" + slot + ",\"attr\":" + ai + ",\"t\":\"OBJECT\"}";
        }
        return "{\"op\":\"var\",\"slot\":" + slot + ",\"chain\":" + chain + ",\"attr\":" + ai + ",\"t\":\"" + lastType
                + "\"}";
    }

    private boolean hasAttr(String stream, String attr) {
        for (Attribute a : streams.get(stream)) {
            if (a.getName().equals(attr)) {
                return true;
            }
        }
        return false;
    }

    private int attrIndex(String stream, String attr) {
        List<Attribute> as = streams.get(stream);
        if (as == null) {
            throw new UnsupportedOnGpuException("stream " + stream + " is not defined");
        }
        for (int i = 0; i < as.size(); i++) {
            if (as.get(i).getName().equals(attr)) {
                return i;
            }
        }
        throw new UnsupportedOnGpuException("attribute " + attr + " not in " + stream);
    }

    private static String str(String s) {
        if (s == null) {
            return "null";
        }
        StringBuilder b = new StringBuilder("\"");
        for (char c : s.toCharArray()) {
            if (c == '"' || c == '\\') {
                b.append('\\').append(c);
            } else if (c < 0x20) {
                b.append(String.format("\\u%04x", (int) c));
            } else {
                b.append(c);
            }
        }
        return b.append('"').toString();
    }
}
