package edu.cmu.reedsolomon;

import java.nio.ByteBuffer;

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

    /**
     * The padded shard length of a file (ReedSolomonEncoder.pad,
     * ReedSolomonEncoder.java:76-85): the file padded with zeros to a multiple
     * of dataShardCount * blockSize, divided by dataShardCount.
     */
    public int shardLengthForFile(int fileLength, int blockSize) {
        if (blockSize < 1) throw new IllegalArgumentException("block size must be positive");
        long mult = (long) dataShardCount * blockSize;
        long padded = fileLength % mult == 0 ? fileLength : (fileLength / mult + 1) * mult;
        return (int) (padded / dataShardCount);
    }

    /**
     * ReedSolomonEncoder.encode() (ReedSolomonEncoder.java:56-74): pads the
     * file, splits it into blockSize-byte blocks round-robin over the data
     * shards (block b to shard b % k at (b / k) * blockSize) and encodes the
     * parity.  The split runs in the native library, so only the file and the
     * parity cross the link.  Returns the k + m shards.
     */
    public byte[][] encodeFile(byte[] fileData, int blockSize) {
        byte[][] shards = new byte[getTotalShardCount()][shardLengthForFile(fileData.length, blockSize)];
        nativeEncodeFile(handle, fileData, blockSize, shards);
        return shards;
    }

    /** encodeFile into caller-allocated shards of at least shardLengthForFile bytes each. */
    public void encodeFile(byte[] fileData, int blockSize, byte[][] shards) {
        nativeEncodeFile(handle, fileData, blockSize, shards);
    }

    /**
     * new ReedSolomonDecoder(shards, shardPresent, byteCntInShard, fileSize)
     * (ReedSolomonDecoder.java:33-39, 62-66, 92-103): decodeMissing(shards,
     * shardPresent, 0, byteCntInShard) in place, then the data shards merged
     * and trimmed to fileSize.  Returns the file.
     */
    public byte[] decodeFile(byte[][] shards, boolean[] shardPresent, int byteCntInShard, int blockSize, int fileSize) {
        byte[] fileData = new byte[fileSize];
        nativeDecodeFile(handle, shards, shardPresent, byteCntInShard, blockSize, fileData, fileSize);
        return fileData;
    }

    /**
     * A direct ByteBuffer over pinned host memory (rs_host_alloc: page-locked,
     * mapped for the GPU, on the calling thread's NUMA node).  Shards and files
     * kept in such buffers are coded in place across the link with no host
     * copies (the ByteBuffer overloads below).  Free it with freePinned; the
     * garbage collector does not.
     */
    public static ByteBuffer allocatePinned(int capacity) {
        return nativeAllocatePinned(capacity);
    }

    /** Frees a buffer from allocatePinned; the buffer must not be used afterwards. */
    public static void freePinned(ByteBuffer buffer) {
        nativeFreePinned(buffer);
    }

    /**
     * encodeParity over direct ByteBuffers (any direct buffer; pinned ones
     * from allocatePinned take the in-place path).  Each shard's length is
     * its capacity; position and limit are ignored.  Same checks, exceptions
     * and messages as the byte[][] form.
     */
    public void encodeParity(ByteBuffer[] shards, int offset, int byteCount) {
        nativeEncodeParityDirect(handle, shards, offset, byteCount);
    }

    /** decodeMissing over direct ByteBuffers (see encodeParity(ByteBuffer[], int, int)). */
    public void decodeMissing(ByteBuffer[] shards, boolean[] shardPresent, int offset, int byteCount) {
        nativeDecodeMissingDirect(handle, shards, shardPresent, offset, byteCount);
    }

    /** encodeFile over direct ByteBuffers: the first fileLength bytes of fileData. */
    public void encodeFile(ByteBuffer fileData, int fileLength, int blockSize, ByteBuffer[] shards) {
        nativeEncodeFileDirect(handle, fileData, fileLength, blockSize, shards);
    }

    /** decodeFile over direct ByteBuffers: fileSize bytes into fileOut. */
    public void decodeFile(ByteBuffer[] shards, boolean[] shardPresent, int byteCntInShard, int blockSize,
                           ByteBuffer fileOut, int fileSize) {
        nativeDecodeFileDirect(handle, shards, shardPresent, byteCntInShard, blockSize, fileOut, fileSize);
    }

    /**
     * Device-resident per-stripe recovery (rs_decode_batch_masked_bits_dev):
     * stripes [stripe][shard][shardStride] at device address devBase, one
     * uint32 presence bitmask per stripe at devBits (bit i = shard i present),
     * asynchronous on the HIP stream handle `stream` (0 = default).  Stripes
     * with fewer than k present shards are skipped and counted into the device
     * int at devBad when it is not 0.  For services that keep chunk groups in
     * GPU memory; the master's host-side loop uses recoverGroupsShardMajor.
     */
    public void decodeMaskedBitsDevice(long devBase, long devBits, long nStripes, long shardLen, long shardStride,
                                       long stripeStride, long devBad, long stream) {
        nativeDecodeMaskedBitsDevice(handle, devBase, devBits, nStripes, shardLen, shardStride, stripeStride, devBad,
                                     stream);
    }

    /**
     * MasterImpl.recoverOfflineChunkserver's loop (MasterImpl.java:794-839)
     * over chunk groups a GPU-side service keeps in HBM in the master's own
     * layout: chunk g of server s at devBase + s * serverStride + g * chunkLen.
     * present holds nGroups * getTotalShardCount() flags, group after group
     * (nonzero: the server answered).  Every absent chunk is rebuilt in place;
     * each run of groups with one offline set is one launch on the given HIP
     * stream (0: the default stream).
     */
    public void recoverGroupsShardMajorDevice(long devBase, long serverStride, int chunkLen, long nGroups,
                                              byte[] present, long stream) {
        nativeRecoverGroupsShardMajorDevice(handle, devBase, serverStride, chunkLen, nGroups, present, stream);
    }

    /**
     * MasterImpl.recoverOfflineChunkserver's loop (MasterImpl.java:733-743,
     * 794-839; ChunkserverDiskRecoveryMachine.java:34-48 per chunk group) on
     * the master's own host arrays, batched: servers[s] holds server s's chunks
     * of nGroups groups back to back (chunk g at g * chunkLen; arrays may be
     * longer), present holds nGroups * getTotalShardCount() flags, group after
     * group (nonzero: the server answered for that group).  Every absent chunk
     * of every group is rebuilt in place from the group's first k present
     * chunks; present chunks are not written.  Instead of one decodeMissing per
     * 6 x 1000-B group, each run of groups with one offline set is ONE decode of
     * run-long shards on the GPU, the arrays pinned only around the library's
     * copy batches.  Throws IllegalArgumentException ("Not enough shards
     * present") before anything is written when a group has fewer than k
     * present.
     */
    public void recoverGroupsShardMajor(byte[][] servers, int chunkLen, int nGroups, byte[] present) {
        nativeRecoverGroupsShardMajor(handle, servers, chunkLen, nGroups, present);
    }

    /** The same over direct buffers (allocatePinned ones are coded in place across the link). */
    public void recoverGroupsShardMajor(ByteBuffer[] servers, int chunkLen, int nGroups, byte[] present) {
        nativeRecoverGroupsShardMajorDirect(handle, servers, chunkLen, nGroups, present);
    }

    /**
     * Frees the calling thread's GPU contexts (HIP streams, device and pinned
     * staging buffers); call from worker threads before a pool retires them.
     */
    public static void releaseThreadResources() {
        nativeThreadRelease();
    }

    @Override
    public synchronized void close() {
        if (handle != 0) {
            nativeDestroy(handle);
            handle = 0;
        }
    }

    private static native long nativeCreate(int k, int m);
    private static native void nativeThreadRelease();
    private static native void nativeDestroy(long h);
    private static native void nativeEncodeParity(long h, byte[][] shards, int offset, int byteCount);
    private static native void nativeDecodeMissing(long h, byte[][] shards, boolean[] present, int offset, int byteCount);
    private static native boolean nativeIsParityCorrect(long h, byte[][] shards, int first, int byteCount, byte[] temp);
    private static native void nativeEncodeFile(long h, byte[] file, int blockSize, byte[][] shards);
    private static native void nativeDecodeFile(long h, byte[][] shards, boolean[] present, int byteCntInShard,
                                                int blockSize, byte[] fileOut, int fileSize);
    private static native ByteBuffer nativeAllocatePinned(int capacity);
    private static native void nativeFreePinned(ByteBuffer buffer);
    private static native void nativeEncodeParityDirect(long h, ByteBuffer[] shards, int offset, int byteCount);
    private static native void nativeDecodeMissingDirect(long h, ByteBuffer[] shards, boolean[] present, int offset,
                                                         int byteCount);
    private static native void nativeEncodeFileDirect(long h, ByteBuffer file, int fileLength, int blockSize,
                                                      ByteBuffer[] shards);
    private static native void nativeDecodeFileDirect(long h, ByteBuffer[] shards, boolean[] present,
                                                      int byteCntInShard, int blockSize, ByteBuffer fileOut,
                                                      int fileSize);
    private static native void nativeDecodeMaskedBitsDevice(long h, long devBase, long devBits, long nStripes,
                                                            long shardLen, long shardStride, long stripeStride,
                                                            long devBad, long stream);
    private static native void nativeRecoverGroupsShardMajorDevice(long h, long devBase, long serverStride,
                                                                   int chunkLen, long nGroups, byte[] present,
                                                                   long stream);
    private static native void nativeRecoverGroupsShardMajor(long h, byte[][] servers, int chunkLen, int nGroups,
                                                             byte[] present);
    private static native void nativeRecoverGroupsShardMajorDirect(long h, ByteBuffer[] servers, int chunkLen,
                                                                   int nGroups, byte[] present);
}
