package edu.cmu.reedsolomon;

/**
 * GPU implementation of the reference's {@code CodingLoop} plugin interface
 * (CodingLoop.java:79-117), for the injection seam
 * {@code new ReedSolomon(k, m, new GpuCodingLoop())} (ReedSolomon.java:37).
 * Results are byte-identical to InputOutputByteTableCodingLoop; the tempBuffer
 * of checkSomeShards is not needed on the GPU and is left untouched.
 */
public final class GpuCodingLoop extends CodingLoopBase {
    static {
        System.loadLibrary("rsamd_jni");
    }

    @Override
    public void codeSomeShards(byte[][] matrixRows, byte[][] inputs, int inputCount,
                               byte[][] outputs, int outputCount, int offset, int byteCount) {
        nativeCodeSomeShards(matrixRows, inputs, inputCount, outputs, outputCount, offset, byteCount);
    }

    @Override
    public boolean checkSomeShards(byte[][] matrixRows, byte[][] inputs, int inputCount,
                                   byte[][] toCheck, int checkCount, int offset, int byteCount,
                                   byte[] tempBuffer) {
        return nativeCheckSomeShards(matrixRows, inputs, inputCount, toCheck, checkCount, offset, byteCount);
    }

    private static native void nativeCodeSomeShards(byte[][] rows, byte[][] inputs, int nin,
                                                    byte[][] outputs, int nout, int offset, int byteCount);
    private static native boolean nativeCheckSomeShards(byte[][] rows, byte[][] inputs, int nin,
                                                        byte[][] toCheck, int ncheck, int offset, int byteCount);
}
