package io.siddhi.gpu;

import io.siddhi.core.config.SiddhiQueryContext;
import io.siddhi.core.stream.StreamJunction;
import io.siddhi.core.util.SiddhiConstants;
import io.siddhi.query.api.SiddhiApp;
import io.siddhi.query.api.execution.query.Query;

import io.siddhi.query.api.definition.Attribute;
import io.siddhi.query.api.definition.StreamDefinition;
import io.siddhi.query.api.util.AnnotationHelper;

import java.util.IdentityHashMap;
import java.util.List;
import java.util.Map;

/**
 * Default provider (META-INF/services/io.siddhi.gpu.PatternRuntimeProvider).  The first query of an app
 * emits the app's descriptor ({@link DescriptorEmitter}) and creates the device runtime; every query then
 * asks it for its path: SG_E_UNSUPPORTED (with {@code sg_query_unsupported_reason}) keeps the stock runtime
 * for that query only.  One receiver per input stream feeds all of the app's device queries (the device
 * dispatches to its subscribers in subscription order, StreamJunction.java:254-272).
 */
public final class GpuRuntimeProvider implements PatternRuntimeProvider {
    private final Map<SiddhiApp, GpuApp> apps = new IdentityHashMap<>();
    private final Map<SiddhiApp, DescriptorEmitter> emitters = new IdentityHashMap<>();

    @Override
    public synchronized GpuQueryRuntime lower(SiddhiApp app, Query query, Map<String, StreamJunction> junctions,
                                              SiddhiQueryContext context) {
        if (Boolean.getBoolean("siddhi.gpu.disable")) {
            return null;
        }
        GpuApp g = apps.get(app);
        DescriptorEmitter em = emitters.get(app);
        if (g == null) {
            String desc;
            em = new DescriptorEmitter(app);
            try {
                desc = em.emit();
            } catch (UnsupportedOnGpuException e) {
                return null;                               // the app uses constructs the descriptor cannot express
            }
            g = new GpuApp(Native.create(desc, Integer.getInteger("siddhi.gpu.device", 0), 0L), junctions,
                    context.getSiddhiAppContext());
            for (Map.Entry<String, List<Attribute>> e : em.allStreams().entrySet()) {
                Attribute.Type[] t = new Attribute.Type[e.getValue().size()];
                for (int i = 0; i < t.length; i++) {
                    t[i] = e.getValue().get(i).getType();
                }
                g.setStreamTypes(Native.streamIndex(g.handle, e.getKey()), t);
            }
            apps.put(app, g);
            emitters.put(app, em);
            g.registerState();
        }
        String name = context.getName();
        for (String s : em.queryInputs.getOrDefault(name, List.of())) {
            // a stream a device query inserts into is also published to its junction for stock consumers; on an
            // @async junction that echo comes back on a worker thread where the receiver cannot tell it from
            // another producer's events, so such a consumer keeps the stock runtime
            if (deviceProduced(g, em, s) && isAsync(app, s)) {
                return null;
            }
        }
        GpuQueryRuntime rt = g.queryRuntime(name, query, em.queryOutStream.get(name), em.queryOutAttrs.get(name));
        if (rt != null) {
            g.setOutputTypes(rt.query, em.queryOutTypes.get(name));
            for (String s : em.queryInputs.get(name)) {
                // every input stream is subscribed, also one a device query inserts into: its other producers (an
                // InputHandler, a source, a stock query) reach the device through the junction, while the events the
                // device query itself produced reach it inside the device (chained dispatch, api.hip) and the
                // receiver drops their junction echo (GpuApp: self-published chunks)
                g.subscribe(s, em.streamAttributes(s));
            }
        }
        return rt;
    }

    private static boolean isAsync(SiddhiApp app, String stream) {
        StreamDefinition d = app.getStreamDefinitionMap().get(stream);
        return d != null && AnnotationHelper.getAnnotation(SiddhiConstants.ANNOTATION_ASYNC, d.getAnnotations()) != null;
    }

    private static boolean deviceProduced(GpuApp g, DescriptorEmitter em, String stream) {
        for (Map.Entry<String, String> e : em.queryOutStream.entrySet()) {
            if (e.getValue().equals(stream) && g.lowered(e.getKey())) {
                return true;
            }
        }
        return false;
    }
}
