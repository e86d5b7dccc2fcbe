/*
 * GpuSketchCommandService -- Redisson's L3 executor (the CommandSyncService of M:Redisson.java:118) serving the
 * probabilistic-structure commands from the MI355X sketch engine.
 *
 * Plugs in at the seam the reference already has: CommandAsyncService.async(...)
 * (M:command/CommandAsyncService.java:378) is the single hook every
 * writeAsync/readAsync goes through; CommandBatchService overrides the same
 * hook to queue (M:command/CommandBatchService.java:91).  It extends
 * CommandSyncService, so Redisson's `CommandExecutor commandExecutor` field
 * (M:Redisson.java:90) takes it as is and the sync read/write/evalRead calls
 * land in the same hook.  Commands for the engine are routed by SketchRouter
 * (shared with the reactive executor, GpuSketchReactiveService); everything
 * else falls through to the Netty -> redis-server path unchanged.  Interfaces
 * in core/ and api/ (RHyperLogLog, RBitSet, RBloomFilter, RBatch) are untouched.
 *
 * Source only here (no JDK in the build image); see INTEGRATION.md.
 */
package org.redisson.gpu;

import java.io.IOException;
import java.nio.charset.Charset;
import java.util.Arrays;
import java.util.HashSet;
import java.util.List;
import java.util.Set;

import org.redisson.client.RedisException;
import org.redisson.client.codec.Codec;
import org.redisson.client.codec.StringCodec;
import org.redisson.client.protocol.DefaultParamsEncoder;
import org.redisson.client.protocol.Encoder;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.client.protocol.RedisCommand.ValueType;
import org.redisson.command.CommandSyncService;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Promise;

public class GpuSketchCommandService extends CommandSyncService implements SketchRouter.RedisPath {

    static final Set<String> SKETCH_COMMANDS = new HashSet<String>(Arrays.asList(
            "PFADD", "PFCOUNT", "PFMERGE", "SETBIT", "GETBIT", "BITCOUNT", "BITOP", "STRLEN"));
    static final Charset UTF8 = Charset.forName("UTF-8");
    /* Generic key commands that act on a sketch key when the engine holds it: RBitSet.toByteArray (GET,
     * M:RedissonBitSet.java:88-91), set(BitSet) (SET, :211-214), clear() / delete() (DEL, :250-253).  The same
     * commands on keys the engine does not hold (RBucket ...) still go to redis-server; DEL is split by holder. */
    static final Set<String> KEY_COMMANDS = new HashSet<String>(Arrays.asList("GET", "SET", "DEL"));
    static final Encoder PARAMS = new DefaultParamsEncoder();

    final long ctx;

    public GpuSketchCommandService(ConnectionManager connectionManager, long ctx) {
        super(connectionManager);
        this.ctx = ctx;
    }

    @Override
    protected <V, R> void async(boolean readOnlyMode, NodeSource source, Codec codec, RedisCommand<V> command,
                                Object[] params, Promise<R> mainPromise, int attempt) {
        if (!SketchRouter.submit(ctx, this, readOnlyMode, source, codec, command, params, mainPromise, attempt)) {
            super.async(readOnlyMode, source, codec, command, params, mainPromise, attempt);
        }
    }

    /** SketchRouter.RedisPath: the reference path (Netty -> redis-server). */
    @Override
    public <V, R> void redisAsync(boolean readOnlyMode, NodeSource source, Codec codec, RedisCommand<V> command,
                                  Object[] params, Promise<R> mainPromise, int attempt) {
        super.async(readOnlyMode, source, codec, command, params, mainPromise, attempt);
    }

    /** The reply convertor the RedisCommand carries (BooleanReplayConvertor, BitSetReplayConvertor ...). */
    static Object convert(RedisCommand<?> command, Object reply) {
        if (command.getConvertor() == null || reply == null) {
            return reply;
        }
        return command.getConvertor().convert(reply);
    }

    /**
     * CommandEncoder.encode's choice of encoder for param i (1-based), M:client/handler/CommandEncoder.java:73-94:
     * with one in-param type, the param AT inParamIndex goes through the codec's value encoder when the type is
     * OBJECT, and params from inParamIndex on go through selectEncoder when it is not; with several types, every
     * param from inParamIndex on goes through selectEncoder(i - inParamIndex); the rest use DefaultParamsEncoder
     * (byte[] as is, else toString() UTF-8).
     */
    static byte[] encodeParam(Codec codec, RedisCommand<?> command, Object param, int i) {
        Encoder encoder = PARAMS;
        List<ValueType> types = command.getInParamType();
        int idx = command.getInParamIndex();
        if (types.size() == 1) {
            if (idx == i && types.get(0) == ValueType.OBJECT) {
                encoder = codec.getValueEncoder();
            } else if (idx <= i && types.get(0) != ValueType.OBJECT) {
                encoder = selectEncoder(codec, types, i - idx);
            }
        } else if (idx <= i) {
            encoder = selectEncoder(codec, types, i - idx);
        }
        try {
            return encoder.encode(param);
        } catch (IOException e) { // what CommandEncoder's caller would surface as a failed command
            throw new RedisException("failed to encode param " + i + " of " + command.getName(), e);
        }
    }

    /** CommandEncoder.selectEncoder, M:client/handler/CommandEncoder.java:101-130. */
    static Encoder selectEncoder(Codec codec, List<ValueType> types, int param) {
        int typeIndex = types.size() > 1 ? param : 0;
        ValueType t = types.get(typeIndex);
        if (t == ValueType.MAP) {
            return param % 2 != 0 ? codec.getMapValueEncoder() : codec.getMapKeyEncoder();
        }
        if (t == ValueType.MAP_KEY) {
            return codec.getMapKeyEncoder();
        }
        if (t == ValueType.MAP_VALUE) {
            return codec.getMapValueEncoder();
        }
        if (t == ValueType.OBJECTS || t == ValueType.OBJECT) {
            return codec.getValueEncoder();
        }
        if (t == ValueType.STRING) {
            return StringCodec.INSTANCE.getValueEncoder();
        }
        throw new IllegalStateException();
    }
}
