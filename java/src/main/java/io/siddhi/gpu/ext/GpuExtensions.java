package io.siddhi.gpu.ext;

import io.siddhi.core.SiddhiManager;

/**
 * Registers the native windows and aggregators under the built-ins' names.  SiddhiManager.setExtension
 * (CORE/SiddhiManager.java:223-229) replaces a built-in with a warning; the extension holders rebuild
 * their cache only when the map's size changes (WindowProcessorExtensionHolder.java:39-43), so call this
 * before the first createSiddhiAppRuntime.
 */
public final class GpuExtensions {
    private GpuExtensions() {
    }

    public static void register(SiddhiManager manager) {
        manager.setExtension("length", GpuWindowProcessors.Length.class);
        manager.setExtension("time", GpuWindowProcessors.Time.class);
        manager.setExtension("lengthBatch", GpuWindowProcessors.LengthBatch.class);
        manager.setExtension("sum", GpuAttributeAggregators.Sum.class);
        manager.setExtension("avg", GpuAttributeAggregators.Avg.class);
        manager.setExtension("count", GpuAttributeAggregators.Count.class);
        manager.setExtension("min", GpuAttributeAggregators.Min.class);
        manager.setExtension("max", GpuAttributeAggregators.Max.class);
    }
}
