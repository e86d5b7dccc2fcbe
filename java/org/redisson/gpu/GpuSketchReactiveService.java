/*
 * GpuSketchReactiveService -- RedissonReactive's L3 executor on the sketch engine.
 *
 * RedissonReactive builds one CommandReactiveService (M:RedissonReactive.java:106), which extends
 * CommandAsyncService (M:command/CommandReactiveService.java:35): every writeReactive / readReactive /
 * evalReadReactive of RHyperLogLogReactive and RBitSetReactive (M:reactive/RedissonHyperLogLogReactive.java,
 * M:reactive/RedissonBitSetReactive.java, which wraps a RedissonBitSet on the same executor) ends in
 * CommandAsyncService.async, and the Publisher is a NettyFuturePublisher over the promise that call completes.
 * This subclass overrides that hook exactly as GpuSketchCommandService does, through the shared SketchRouter:
 * engine commands run on the context's FIFO worker and complete the promise there (the subscriber's onNext runs
 * from that completion), everything else goes to redis-server through super.async.  RBatchReactive's executor is
 * a CommandBatchService (M:reactive/RedissonBatchReactive.java:51), which GpuSketchBatchService replaces.
 * Source only here; see INTEGRATION.md.
 */
package org.redisson.gpu;

import org.redisson.client.codec.Codec;
import org.redisson.client.protocol.RedisCommand;
import org.redisson.command.CommandReactiveService;
import org.redisson.connection.ConnectionManager;
import org.redisson.connection.NodeSource;

import io.netty.util.concurrent.Promise;

public class GpuSketchReactiveService extends CommandReactiveService implements SketchRouter.RedisPath {

    final long ctx;

    public GpuSketchReactiveService(ConnectionManager connectionManager, long ctx) {
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
}
