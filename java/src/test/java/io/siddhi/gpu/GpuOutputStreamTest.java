package io.siddhi.gpu;

import io.siddhi.core.SiddhiAppRuntime;
import io.siddhi.core.SiddhiManager;
import io.siddhi.core.event.Event;
import io.siddhi.core.stream.input.InputHandler;
import io.siddhi.core.stream.output.StreamCallback;
import io.siddhi.core.util.EventPrinter;
import org.testng.Assert;
import org.testng.annotations.Test;

import java.util.ArrayList;
import java.util.List;

/**
 * The device provider on the class path (META-INF/services), siddhi-core patched with
 * java/patches/siddhi-core-external-query-runtime.patch: a StreamCallback on the `insert into` stream of a
 * device query that was never declared receives its output, a stock query reading that stream sees it, and the
 * state survives snapshot / restore.  (Needs a JDK and the siddhi jars: not built in this repository's image.)
 */
public class GpuOutputStreamTest {

    private static final String APP = "@app:playback define stream StockStream (symbol string, price float, volume int); "
            + "@info(name = 'query1') from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] "
            + "within 1 sec select e1.symbol as symbol, e2.price as price insert into Matches; "
            + "@info(name = 'query2') from Matches[price > 50] select symbol insert into High;";

    @Test
    public void undeclaredOutputStreamReachesStreamCallbacks() throws InterruptedException {
        SiddhiManager manager = new SiddhiManager();
        SiddhiAppRuntime runtime = manager.createSiddhiAppRuntime(APP);
        List<Event> matches = new ArrayList<>();
        List<Event> high = new ArrayList<>();
        runtime.addCallback("Matches", new StreamCallback() {
            @Override
            public void receive(Event[] events) {
                EventPrinter.print(events);
                for (Event e : events) {
                    matches.add(e);
                }
            }
        });
        runtime.addCallback("High", new StreamCallback() {
            @Override
            public void receive(Event[] events) {
                for (Event e : events) {
                    high.add(e);
                }
            }
        });
        runtime.start();
        InputHandler in = runtime.getInputHandler("StockStream");
        in.send(1000L, new Object[]{"A", 30f, 1});
        in.send(1100L, new Object[]{"A", 60f, 1});
        byte[] state = runtime.snapshot();
        in.send(1200L, new Object[]{"A", 70f, 1});
        runtime.restore(state);
        in.send(1300L, new Object[]{"A", 75f, 1});
        runtime.shutdown();
        // 60 completes 30; after the restore 60 is pending again and 75 completes it (70 was rolled back)
        Assert.assertEquals(matches.size(), 3);
        Assert.assertEquals(high.size(), 3);
        manager.shutdown();
    }

    /**
     * A stream with two producers: a device query inserts into Matches and an InputHandler sends to Matches
     * directly.  The device consumer (query2) must see both: the device query's rows inside the device, the
     * InputHandler's through the junction -- and the junction echo of the device's own rows exactly once.
     */
    @Test
    public void deviceAndInputHandlerFeedOneStream() throws InterruptedException {
        SiddhiManager manager = new SiddhiManager();
        SiddhiAppRuntime runtime = manager.createSiddhiAppRuntime(APP);
        List<Event> high = new ArrayList<>();
        runtime.addCallback("High", new StreamCallback() {
            @Override
            public void receive(Event[] events) {
                for (Event e : events) {
                    high.add(e);
                }
            }
        });
        runtime.start();
        InputHandler stock = runtime.getInputHandler("StockStream");
        InputHandler direct = runtime.getInputHandler("Matches");
        stock.send(1000L, new Object[]{"A", 30f, 1});
        stock.send(1100L, new Object[]{"A", 60f, 1});      // device match (A, 60) -> High
        direct.send(1200L, new Object[]{"B", 90f});         // direct row (B, 90) -> High
        direct.send(1300L, new Object[]{"C", 10f});         // filtered out by query2
        runtime.shutdown();
        Assert.assertEquals(high.size(), 2);
        Assert.assertEquals(high.get(0).getData()[0], "A");
        Assert.assertEquals(high.get(1).getData()[0], "B");
        manager.shutdown();
    }

    /**
     * Re-entrant drain: device query1 publishes Matches; the stock query2 (a function executor keeps it off the
     * device) inserts every Matches row into Back synchronously, and the device query3 reads Back, so its push
     * re-enters the drain on the publishing thread.  The device query4 is a second consumer of Matches behind
     * query2 in the junction's receiver list: the nested drain must not clear the outer publish's echo marker, or
     * query4 would receive each device row twice.
     */
    @Test
    public void nestedDrainKeepsEchoSuppression() throws InterruptedException {
        String app = "@app:playback define stream StockStream (symbol string, price float, volume int); "
                + "@info(name = 'query1') from every e1=StockStream[price > 20] -> e2=StockStream[price > e1.price] "
                + "within 1 sec select e1.symbol as symbol, e2.price as price insert into Matches; "
                + "@info(name = 'query2') from Matches select symbol, cast(price, 'float') as price insert into Back; "
                + "@info(name = 'query3') from Back[price > 0] select symbol, price insert into Echoed; "
                + "@info(name = 'query4') from Matches[price > 50] select symbol insert into High;";
        SiddhiManager manager = new SiddhiManager();
        SiddhiAppRuntime runtime = manager.createSiddhiAppRuntime(app);
        List<Event> high = new ArrayList<>();
        List<Event> echoed = new ArrayList<>();
        runtime.addCallback("High", new StreamCallback() {
            @Override
            public void receive(Event[] events) {
                for (Event e : events) {
                    high.add(e);
                }
            }
        });
        runtime.addCallback("Echoed", new StreamCallback() {
            @Override
            public void receive(Event[] events) {
                for (Event e : events) {
                    echoed.add(e);
                }
            }
        });
        runtime.start();
        InputHandler stock = runtime.getInputHandler("StockStream");
        stock.send(1000L, new Object[]{"A", 30f, 1});
        stock.send(1100L, new Object[]{"A", 60f, 1});      // (A, 60): Matches -> Back -> Echoed, and High
        stock.send(1200L, new Object[]{"A", 70f, 1});      // (A, 70) completes the start at 60
        runtime.shutdown();
        Assert.assertEquals(echoed.size(), 2);
        Assert.assertEquals(high.size(), 2);
        manager.shutdown();
    }
}
