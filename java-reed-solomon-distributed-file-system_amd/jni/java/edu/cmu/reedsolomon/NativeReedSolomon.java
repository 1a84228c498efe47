package edu.cmu.reedsolomon;

/**
 * GPU-backed drop-in for {@code ReedSolomon} (ReedSolomon.java:13-344 of the
 * reference): same factory, getters and coding methods, same exceptions and
 * messages, shards mutated in place.  Every byte is coded by the MI355X kernels
 * of librsamd.so through librsamd_jni.so (rs_jni.c).
 *
 * Decode is one GPU pass (the reference runs two codeSomeShards passes); the
 * reconstructed bytes are identical (DESIGN.md section 3.3).
 */
public final class NativeReedSolomon implements AutoCloseable {
    static {
        System.loadLibrary("rsamd_jni");
    }

    private final int dataShardCount;
    private final int parityShardCount;
    private long handle;

    public static NativeReedSolomon create(int dataShardCount, int parityShardCount) {
        return new NativeReedSolomon(dataShardCount, parityShardCount);
    }

    public NativeReedSolomon(int dataShardCount, int parityShardCount) {
        this.handle = nativeCreate(dataShardCount, parityShardCount);  // throws IAE like ReedSolomon.java:44-46
        this.dataShardCount = dataShardCount;
        this.parityShardCount = parityShardCount;
    }

    public int getDataShardCount() { return dataShardCount; }
    public int getParityShardCount() { return parityShardCount; }
    public int getTotalShardCount() { return dataShardCount + parityShardCount; }

    public void encodeParity(byte[][] shards, int offset, int byteCount) {
        nativeEncodeParity(handle, shards, offset, byteCount);
    }

    public boolean isParityCorrect(byte[][] shards, int firstByte, int byteCount) {
        return nativeIsParityCorrect(handle, shards, firstByte, byteCount, null);
    }

    public boolean isParityCorrect(byte[][] shards, int firstByte, int byteCount, byte[] tempBuffer) {
        if (tempBuffer == null) throw new NullPointerException();  // the reference reads tempBuffer.length
        return nativeIsParityCorrect(handle, shards, firstByte, byteCount, tempBuffer);
    }

    public void decodeMissing(byte[][] shards, boolean[] shardPresent, int offset, int byteCount) {
        nativeDecodeMissing(handle, shards, shardPresent, offset, byteCount);
    }

    @Override
    public synchronized void close() {
        if (handle != 0) {
            nativeDestroy(handle);
            handle = 0;
        }
    }

    private static native long nativeCreate(int k, int m);
    private static native void nativeDestroy(long h);
    private static native void nativeEncodeParity(long h, byte[][] shards, int offset, int byteCount);
    private static native void nativeDecodeMissing(long h, byte[][] shards, boolean[] present, int offset, int byteCount);
    private static native boolean nativeIsParityCorrect(long h, byte[][] shards, int first, int byteCount, byte[] temp);
}
