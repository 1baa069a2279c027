// Type declarations for lodestar_amd/js/bls_gpu_verifier.js: the GPU verifier as a
// Lodestar IBlsVerifier (packages/beacon-node/src/chain/bls/interface.ts:4-68), so a
// TypeScript beacon node can construct it where chain.ts:206-208 picks the bls pool.
// Signature sets follow @lodestar/state-transition's ISignatureSet
// (packages/state-transition/src/util/signatureSets.ts:5-24); a pubkey may be given by
// validator index ({index}) once syncPubkeys() has mirrored index2pubkey on the GPUs.

/** @chainsafe/bls PointFormat (the reference serializes with PointFormat.uncompressed,
 * BN/chain/bls/multithread/index.ts:144 -> jobItem.ts:59). */
export type PointFormat = "compressed" | "uncompressed";
export const PointFormat: {compressed: "compressed"; uncompressed: "uncompressed"};
/** The shape of a @chainsafe/bls PublicKey this verifier needs: toBytes(format) returns the
 * compressed 48-byte encoding unless format is "uncompressed" (96 bytes). */
export type PublicKeyLike = {toBytes(format?: PointFormat): Uint8Array};
/** A public key: a @chainsafe/bls PublicKey (as index2pubkey holds them; shipped as its
 * validator index once syncPubkeys/syncIndex2pubkey mirrored it, else serialized with
 * toBytes("uncompressed")), its 96-byte uncompressed or 48-byte compressed encoding, or
 * {index}: a validator index into the GPUs' pubkey tables. */
export type GpuPublicKey = PublicKeyLike | Uint8Array | {index: number};

/** signatureSets.ts:5-24 */
export type SingleSignatureSet = {
  type: "single";
  pubkey: GpuPublicKey;
  signingRoot: Uint8Array;
  signature: Uint8Array;
};
export type AggregatedSignatureSet = {
  type: "aggregate";
  pubkeys: GpuPublicKey[];
  signingRoot: Uint8Array;
  signature: Uint8Array;
};
export type ISignatureSet = SingleSignatureSet | AggregatedSignatureSet;

/** interface.ts:4-23 */
export type VerifySignatureOpts = {
  batchable?: boolean;
  /** here: the device's priority lane at once (no queue, no JS main-thread blocking) */
  verifyOnMainThread?: boolean;
  /** here: queue front, then the device's priority lane (lb_verify_requests_priority_async) */
  priority?: boolean;
};

/** interface.ts:25-75 */
export interface IBlsVerifier {
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  verifySignatureSetsSameMessage(
    sets: {publicKey: GpuPublicKey; signature: Uint8Array}[],
    message: Uint8Array,
    opts?: Omit<VerifySignatureOpts, "verifyOnMainThread">
  ): Promise<boolean[]>;
  close(): Promise<void>;
  canAcceptWork(): boolean;
}

/** The addon's batch (include/lodestar_bls.h lb_request_batch). */
export type PackedRequests = {
  requestOffsets: Uint32Array;
  pkOffsets?: Uint32Array;
  pubkeys?: Uint8Array;
  pubkeyIndices?: Uint32Array;
  messages: Uint8Array;
  signatures: Uint8Array;
  sigOffsets: Uint32Array;
  seed: Uint8Array;
  batchable?: Uint8Array;
};

export type SameMessageBatch = {
  jobOffsets: Uint32Array;
  pubkeys?: Uint8Array;
  pubkeyIndices?: Uint32Array;
  signatures: Uint8Array;
  sigOffsets: Uint32Array;
  messages: Uint8Array;
  seed: Uint8Array;
};

export type VerifyResult = {
  valid: Uint8Array;
  errors: Uint8Array;
  setStatus: Uint8Array;
  batchRetries: number;
  batchSigsSuccess: number;
  deviceMs: number;
  workerStartNs?: number;
  workerEndNs?: number;
};

/** One GPU: the N-API addon's Context (lodestar_amd/napi/addon.cc), or a mock. */
export interface GpuBackend {
  capacity?: number;
  verifyRequests(batch: PackedRequests, opts?: {priority?: boolean}): Promise<VerifyResult>;
  verifyRequestsPartial?(batch: PackedRequests): Promise<{id: number; partial: Uint8Array}>;
  finish?(id: number, mergedOk: boolean): Promise<VerifyResult>;
  gtCheck?(partials: Uint8Array): Promise<boolean>;
  verifySameMessage(batch: SameMessageBatch): Promise<{
    valid: Uint8Array;
    jobFast: Uint8Array;
    retriedJobs: number;
    fastSets: number;
    deviceMs: number;
  }>;
  syncPubkeys?(keys: Uint8Array, pkLen: number): Promise<number>;
  aggregatePubkeys?(keys: Uint8Array | Uint32Array): Promise<Uint8Array>;
  close?(): Promise<void>;
}

export type BlsGpuVerifierOpts = {
  /** GPU ordinals, one addon Context each (default [0]) */
  devices?: number[];
  /** Context-like objects instead (tests: mocks) */
  backends?: GpuBackend[];
  /** calls in flight per GPU (default: the library's lb_slots) */
  capacity?: number;
  blsVerifyAllMultiThread?: boolean;
  maxSetsPerDispatch?: number;
  prefetch?: number;
  seedSource?: () => Uint8Array;
  /** priority jobs and verifyOnMainThread calls take the device's priority lane (default true) */
  priorityLane?: boolean;
};

/** BlsMultiThreadWorkerPool (chain/bls/multithread/index.ts) on GPUs. */
export class BlsGpuVerifier implements IBlsVerifier {
  constructor(opts?: BlsGpuVerifierOpts);
  readonly capacity: number;
  readonly metrics: PoolMetrics;
  /** Append keys to every GPU's pubkey table (pubkeyCache.ts:56-77); PublicKey objects are
   * serialized once here and then ship as their table index.  Returns the table size. */
  syncPubkeys(keys: (Uint8Array | PublicKeyLike)[], pkLen?: 48 | 96): Promise<number>;
  /** pubkeyCache.syncPubkeys for the GPUs: mirror index2pubkey's new entries (incremental);
   * returns the number of entries mirrored. */
  syncIndex2pubkey(index2pubkey: PublicKeyLike[]): Promise<number>;
  verifySignatureSets(sets: ISignatureSet[], opts?: VerifySignatureOpts): Promise<boolean>;
  verifySignatureSetsSameMessage(
    sets: {publicKey: GpuPublicKey; signature: Uint8Array}[],
    message: Uint8Array,
    opts?: Omit<VerifySignatureOpts, "verifyOnMainThread">
  ): Promise<boolean[]>;
  close(): Promise<void>;
  canAcceptWork(): boolean;
}

/** BlsSingleThreadVerifier (chain/bls/singleThread.ts:10-89) on one GPU. */
export class BlsGpuSingleThreadVerifier implements IBlsVerifier {
  constructor(opts?: {backend?: GpuBackend; device?: number; seedSource?: () => Uint8Array; metrics?: PoolMetrics});
  syncPubkeys(keys: (Uint8Array | PublicKeyLike)[], pkLen?: 48 | 96): Promise<number>;
  syncIndex2pubkey(index2pubkey: PublicKeyLike[]): Promise<number>;
  verifySignatureSets(sets: ISignatureSet[]): Promise<boolean>;
  verifySignatureSetsSameMessage(
    sets: {publicKey: GpuPublicKey; signature: Uint8Array}[],
    message: Uint8Array
  ): Promise<boolean[]>;
  close(): Promise<void>;
  canAcceptWork(): boolean;
}

export const QueueErrorCode: {QUEUE_ABORTED: "QUEUE_ERROR_QUEUE_ABORTED"};
export class QueueError extends Error {
  constructor(code: string);
  type: {code: string};
}

/** The reference's metric names (metrics/metrics/lodestar.ts:379-510), kept in-process. */
export class PoolMetrics {
  inc(name: string, v?: number, labels?: Record<string, string | number>): void;
  set(name: string, v: number, labels?: Record<string, string | number>): void;
  observe(name: string, v: number, labels?: Record<string, string | number>): void;
  get(name: string, labels?: Record<string, string | number>): number;
}
export const METRICS: Record<string, string>;

export function chunkifyMaximizeChunkSize<T>(arr: T[], minPerChunk: number): T[][];
export function workerBatchStats(
  requestSizes: number[],
  batchable: boolean[],
  valid: boolean[]
): {retries: number; sigsOk: number};
export function packRequests(
  requests: ISignatureSet[][],
  seed: Uint8Array,
  keyMap?: WeakMap<object, number>
): PackedRequests;
export function packSameMessage(
  jobs: {sets: {publicKey: GpuPublicKey; signature: Uint8Array}[]; message: Uint8Array}[],
  seed: Uint8Array,
  keyMap?: WeakMap<object, number>
): SameMessageBatch;
export function shardRequests(sizes: number[], nShards: number): [number, number][];
export function slicePacked(p: PackedRequests, lo: number, hi: number, seed: Uint8Array): PackedRequests;
/** Several GPUs, one combined final exponentiation over the shards' Fp12 partials. */
export function verifyRequestsSharded(
  backends: GpuBackend[],
  requests: ISignatureSet[][],
  seedSource: () => Uint8Array
): Promise<{valid: Uint8Array; errors: Uint8Array; mergedOk: boolean}>;
export function verifyPackedSharded(
  backends: GpuBackend[],
  packed: PackedRequests,
  seedSource: () => Uint8Array
): Promise<{valid: Uint8Array; errors: Uint8Array; mergedOk: boolean}>;
export function loadAddon(): {
  deviceCount(): number;
  Context: new (device: number, opts?: {capacity?: number}) => GpuBackend;
};

export const MAX_SIGNATURE_SETS_PER_JOB: 128;
export const MAX_BUFFERED_SIGS: 32;
export const MAX_BUFFER_WAIT_MS: 100;
export const MAX_JOBS_CAN_ACCEPT_WORK: 512;
export const MAX_PRIORITY_LANE_SETS: 1024;
/** lb_request_batch / lb_same_message_batch pubkeyIndices flags (include/lodestar_bls.h) */
export const LB_PK_ROW_FLAG: 0x80000000;
export const LB_PK_ROW48_FLAG: 0x40000000;
