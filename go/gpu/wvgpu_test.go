//go:build rocm

package gpu

import (
	"testing"

	"github.com/weaviate/weaviate/adapters/repos/db/helpers"
)

// A non-nil, empty AllowList returns nothing (V/flat/index.go:423-427);
// a nil one searches every row.
func TestEmptyAllowListReturnsNothing(t *testing.T) {
	ctx, err := Open(0)
	if err != nil {
		t.Skip("no GPU:", err)
	}
	defer ctx.Close()
	const n, dims = 1000, 16
	x, err := ctx.NewCorpus(KindF32, MetricL2, dims, 0, n)
	if err != nil {
		t.Fatal(err)
	}
	defer x.Close()
	ids := make([]uint64, n)
	rows := make([]float32, n*dims)
	for i := range ids {
		ids[i] = uint64(i)
		for j := 0; j < dims; j++ {
			rows[i*dims+j] = float32((i*31+j*7)%97) / 97
		}
	}
	if err := x.Add(ids, rows); err != nil {
		t.Fatal(err)
	}
	q := rows[:dims]
	got, _, err := x.Search(q, 10, helpers.NewAllowList())
	if err != nil || len(got) != 0 {
		t.Fatalf("empty allow list: %v results, err %v", len(got), err)
	}
	got, d, err := x.Search(q, 10, nil)
	if err != nil || len(got) != 10 || got[0] != 0 || d[0] != 0 {
		t.Fatalf("nil allow list: %v %v %v", got, d, err)
	}
	got, _, err = x.Search(q, 10, helpers.NewAllowList(5, 7))
	if err != nil || len(got) != 2 {
		t.Fatalf("allow list {5, 7}: %v %v", got, err)
	}
}
