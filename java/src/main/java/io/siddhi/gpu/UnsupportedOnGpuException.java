package io.siddhi.gpu;

/** SG_E_UNSUPPORTED: the device has no lowering for this query or input; the stock runtime keeps it. */
public class UnsupportedOnGpuException extends RuntimeException {
    public UnsupportedOnGpuException(String message) {
        super(message);
    }
}
